// crc32c_multi.hip -- several GPUs of one node (include/hdfs_crc32c.h
// section 5): a file's packets dealt round-robin over the GPUs in groups of
// consecutive packets (one HDFS block each: fuse.c:580-647 writes a file
// block by block, hadoop_rpc_send_packets cuts each block into packets,
// hadooprpc.c:815-860), every GPU checksumming its shard device-resident,
// and one RCCL group of point-to-point transfers over xGMI gathering the
// u32 checksum arrays into block order on rank 0's device.  The checksums
// are the path's only exchange; no payload byte crosses GPUs.
//
// Rank 0 checksums its own groups straight into their final places; every
// other rank checksums its groups into one local array.  When each sender's
// groups land in one file-order range (contiguous sharding, or N = 1), it
// sends that range with one ncclSend and rank 0 receives it straight into
// place.  When a sender's groups are spread over the file (round-robin
// blocks: at N = 8 a rank's 4 blocks are 8 blocks apart), it still sends its
// whole local array with ONE ncclSend, into a staging array on rank 0, and
// one scatter kernel on rank 0 moves every group's range into file order:
// point-to-point operations in one RCCL group are served one after another
// per peer, each at a fixed cost (one GPU: a 16 MiB shard step 12.9 us with
// one self-send, 34.7 us with four), so one operation
// per peer plus a 1 MiB copy beats one per group.  CRC32C_MULTI_PER_GROUP_RECV
// keeps one operation per group range (A/B).  (A one-GPU communicator needs
// no transfer; CRC32C_MULTI_SELF_SEND routes rank 0's own checksums through
// RCCL as well, to exercise the transport on one GPU.)
//
// Two ways to build the communicator: one process driving every device
// (crc32c_multi_create, ncclCommInitAll) or one process per device
// (crc32c_multi_create_rank, ncclCommInitRank with an id from
// crc32c_multi_unique_id passed between the processes by the caller).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <type_traits>
#include <vector>

#include "hdfs_crc32c.h"
#include "plan.h"
#include "runtime_internal.h"

using namespace hdfs_crc;

// RCCL is loaded on first use (dlopen by SONAME, so a process that already
// holds torch's RCCL shares it), not linked: a single-GPU caller of the
// library -- the FUSE daemon's write path -- needs no RCCL at load time.
namespace {

struct Rccl {
    decltype(&ncclGetUniqueId) GetUniqueId = nullptr;
    decltype(&ncclCommInitRank) CommInitRank = nullptr;
    decltype(&ncclCommInitAll) CommInitAll = nullptr;
    decltype(&ncclCommDestroy) CommDestroy = nullptr;
    decltype(&ncclGroupStart) GroupStart = nullptr;
    decltype(&ncclGroupEnd) GroupEnd = nullptr;
    decltype(&ncclSend) Send = nullptr;
    decltype(&ncclRecv) Recv = nullptr;
    decltype(&ncclGetErrorString) GetErrorString = nullptr;
    std::string error;
};

const Rccl &rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        void *h = nullptr;
        for (const char *name : {"librccl.so.1", "librccl.so"})
            if ((h = dlopen(name, RTLD_NOW | RTLD_GLOBAL))) break;
        if (!h) {
            const char *e = dlerror();
            r.error = e ? e : "librccl.so.1 not found";
            return;
        }
        bool ok = true;
        auto sym = [&](auto &fn, const char *name) {
            fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
            ok = ok && fn;
        };
        sym(r.GetUniqueId, "ncclGetUniqueId");
        sym(r.CommInitRank, "ncclCommInitRank");
        sym(r.CommInitAll, "ncclCommInitAll");
        sym(r.CommDestroy, "ncclCommDestroy");
        sym(r.GroupStart, "ncclGroupStart");
        sym(r.GroupEnd, "ncclGroupEnd");
        sym(r.Send, "ncclSend");
        sym(r.Recv, "ncclRecv");
        sym(r.GetErrorString, "ncclGetErrorString");
        if (!ok) {
            r.error = "librccl is missing a symbol";
            r.GetUniqueId = nullptr;
        }
    });
    return r;
}

}  // namespace

#define RCCL_LOADED()                                                                          \
    do {                                                                                       \
        if (!rccl().GetUniqueId) return fail(-ENOSYS, "RCCL unavailable: %s", rccl().error.c_str()); \
    } while (0)

#define NCCL_TRY(expr)                                                                                  \
    do {                                                                                                \
        ncclResult_t r_ = (expr);                                                                       \
        if (r_ != ncclSuccess)                                                                          \
            return fail(-EIO, "%s: %s (%s:%d)", #expr, rccl().GetErrorString(r_), __FILE__, __LINE__);  \
    } while (0)

struct crc32c_multi {
    std::vector<crc32c_ctx *> ctxs;  // local devices
    std::vector<int> ranks;          // communicator rank of each local device
    int nranks = 0;
    std::vector<ncclComm_t> comms;   // per local device (single-process: created on first exec)
    std::vector<hipStream_t> streams;  // per local device, used when the caller passes none
    std::mutex mu;
};

namespace {

// One group of consecutive packets (an HDFS block) and where it lives.
struct Group {
    uint64_t lo = 0, hi = 0;  // payload range of its non-empty packets in the caller's layout
    uint64_t omin = 0, n = 0;  // its checksums: global out indices [omin, omin + n)
    int rank = 0;
    uint64_t shard_off = 0;  // where byte lo sits in its rank's shard (same 16-byte phase)
    uint64_t local_out = 0;  // index of its first checksum in its rank's local array
};

// Groups of `gp` packets, group g on rank g % nranks; each rank's shard is
// its groups' byte ranges back to back (16-byte phase kept), its local
// checksum array their checksum ranges back to back.
int build_layout(const crc32c_packet *pkts, size_t npkts, uint32_t gp, int nranks, std::vector<Group> *groups,
                 std::vector<uint64_t> *shard_bytes, std::vector<uint64_t> *local_nout) {
    if (nranks <= 0 || gp == 0 || (npkts && !pkts)) return fail(-EINVAL, "bad layout arguments");
    groups->assign((npkts + gp - 1) / gp, Group());
    shard_bytes->assign(size_t(nranks), 0);
    local_nout->assign(size_t(nranks), 0);
    for (size_t g = 0; g < groups->size(); ++g) {
        Group &G = (*groups)[g];
        uint64_t lo = UINT64_MAX, hi = 0, n = 0;
        std::vector<std::pair<uint64_t, uint64_t>> outs;  // (out_idx, checksums) of its packets
        for (size_t i = g * gp; i < std::min<size_t>(npkts, (g + 1) * gp); ++i) {
            const crc32c_packet &p = pkts[i];
            if (!p.len) continue;  // (no checksums, whatever its bpc)
            if (p.bpc == 0) return fail(-EINVAL, "packet %zu: bytesPerChecksum == 0", i);
            const uint64_t c = crc32c_nchunks(p.len, p.bpc);
            lo = std::min(lo, p.payload_off);
            hi = std::max(hi, p.payload_off + p.len);
            outs.emplace_back(p.out_idx, c);
            n += c;
        }
        G.rank = int(g % size_t(nranks));
        if (lo == UINT64_MAX) continue;  // only empty packets
        // its packets' checksum ranges must tile one contiguous range
        std::sort(outs.begin(), outs.end());
        for (size_t k = 1; k < outs.size(); ++k)
            if (outs[k].first != outs[k - 1].first + outs[k - 1].second)
                return fail(-EINVAL, "group %zu: its checksums are not one contiguous range", g);
        const uint64_t omin = outs.front().first;
        G.lo = lo;
        G.hi = hi;
        G.omin = omin;
        G.n = n;
        uint64_t &cur = (*shard_bytes)[size_t(G.rank)];
        G.shard_off = ((cur + 15) & ~uint64_t(15)) + (lo & 15);
        cur = G.shard_off + (hi - lo);
        G.local_out = (*local_nout)[size_t(G.rank)];
        (*local_nout)[size_t(G.rank)] += n;
    }
    return 0;
}

// Rank r's packets: payload offsets in its shard; out indices in its local
// array (local = true) or the global ones.
void shard_packets(const crc32c_packet *pkts, size_t npkts, uint32_t gp, const std::vector<Group> &groups, int rank,
                   bool local, std::vector<crc32c_packet> *out) {
    out->clear();
    for (size_t g = 0; g < groups.size(); ++g) {
        const Group &G = groups[g];
        if (G.rank != rank) continue;
        for (size_t i = g * gp; i < std::min<size_t>(npkts, (g + 1) * gp); ++i) {
            crc32c_packet p = pkts[i];
            if (!p.len) continue;
            p.payload_off = G.shard_off + (p.payload_off - G.lo);
            if (local) p.out_idx = G.local_out + (p.out_idx - G.omin);
            out->push_back(p);
        }
    }
}

// The gather step of a plan: the point-to-point transfers, in the order they
// are posted -- {sending rank, index in its local array, file index on rank
// 0, count}.  One per received group, merged with the previous one when both
// come from the same rank and stay contiguous on both sides (a one-rank
// self-send is then one transfer).  Every sender posts its ncclSends and rank
// 0 its ncclRecvs (straight into the file-order output) in this order, so
// each (sender, rank 0) pair matches in order.  Rank 0's own groups are
// computed in place (no transfer) unless self_send.  crc32c_multi_plan_create
// builds its exec from exactly this; crc32c_multi_transfers exports it.
struct Xfer {
    int rank;
    uint64_t local, file, count;
};
// Transfers one exec's RCCL group may hold (crc32c_multi_plan_create refuses more).
constexpr size_t kMaxGatherTransfers = 4096;

bool sends(int rank, bool self_send) { return rank != 0 || self_send; }

void build_transfers(const std::vector<Group> &groups, bool self_send, std::vector<Xfer> *xs) {
    xs->clear();
    for (const Group &G : groups) {
        if (!G.n || !sends(G.rank, self_send)) continue;
        if (!xs->empty()) {
            Xfer &b = xs->back();
            if (b.rank == G.rank && b.local + b.count == G.local_out && b.file + b.count == G.omin) {
                b.count += G.n;
                continue;
            }
        }
        xs->push_back(Xfer{G.rank, G.local_out, G.omin, G.n});
    }
}

// The packed gather (one operation per sender): rank r's whole local array
// lands at stage_off[r] of rank 0's staging array; the scatter kernel then
// copies each group range into file order, in tiles of at most kScatterTile
// checksums (one workgroup each).
struct ScatterTile {
    uint32_t src, dst, n, pad;
};
constexpr uint32_t kScatterTile = 1024;  // (4 per thread: one load round trip per workgroup)

// true when some sender has more than one group range (placement) to send.
bool wants_packed(const std::vector<Xfer> &xs) {
    for (size_t k = 1; k < xs.size(); ++k)
        for (size_t j = 0; j < k; ++j)
            if (xs[j].rank == xs[k].rank) return true;
    return false;
}

// Where each sender's local array lands in rank 0's staging array (rank
// order); returns the staging array's length.
uint64_t stage_offsets(const std::vector<uint64_t> &local_nout, bool self_send, std::vector<uint64_t> *stage_off) {
    uint64_t n = 0;
    stage_off->assign(local_nout.size(), 0);
    for (size_t q = 0; q < local_nout.size(); ++q)
        if (sends(int(q), self_send)) {
            (*stage_off)[q] = n;
            n += local_nout[q];
        }
    return n;
}

void build_scatter(const std::vector<Xfer> &xs, const std::vector<uint64_t> &stage_off,
                   std::vector<ScatterTile> *tiles) {
    tiles->clear();
    for (const Xfer &x : xs)
        for (uint64_t o = 0; o < x.count; o += kScatterTile)
            tiles->push_back(ScatterTile{uint32_t(stage_off[size_t(x.rank)] + x.local + o), uint32_t(x.file + o),
                                         uint32_t(std::min<uint64_t>(kScatterTile, x.count - o)), 0u});
}

__global__ __launch_bounds__(256) void hdfs_crc32c_gather_scatter(const uint32_t *__restrict__ stage,
                                                                 uint32_t *__restrict__ out,
                                                                 const ScatterTile *__restrict__ tiles) {
    const ScatterTile t = tiles[blockIdx.x];
    uint32_t v[4];
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) {
        const uint32_t k = threadIdx.x + 256u * j;
        v[j] = k < t.n ? stage[t.src + k] : 0u;
    }
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) {
        const uint32_t k = threadIdx.x + 256u * j;
        if (k < t.n) out[t.dst + k] = v[j];
    }
}

// The packets rank r's plan computes: payload offsets in its shard; out
// indices in its local array, or the global ones when rank 0 works in place.
void rank_plan_packets(const crc32c_packet *pkts, size_t npkts, uint32_t gp, const std::vector<Group> &groups, int r,
                       bool self_send, std::vector<crc32c_packet> *out) {
    shard_packets(pkts, npkts, gp, groups, r, sends(r, self_send), out);
}

int ensure_comms(crc32c_multi *m) {
    if (!m->comms.empty()) return 0;
    std::vector<int> devs;
    for (crc32c_ctx *c : m->ctxs) devs.push_back(c->device);
    std::vector<ncclComm_t> comms(devs.size());
    RCCL_LOADED();
    NCCL_TRY(rccl().CommInitAll(comms.data(), int(devs.size()), devs.data()));
    m->comms = comms;
    return 0;
}

// The caller's stream of local device i (NULL = that device's default
// stream), or the library's own when the caller passes no stream array.
hipStream_t local_stream(crc32c_multi *m, size_t i, void *const *streams) {
    if (streams) return static_cast<hipStream_t>(streams[i]);
    return m->streams[i];
}

}  // namespace

struct crc32c_multi_plan {
    crc32c_multi *m = nullptr;
    std::vector<Group> groups;
    std::vector<uint64_t> shard_bytes;  // per rank
    std::vector<uint64_t> local_nout;   // per rank: checksums of its shard
    std::vector<crc32c_plan *> plans;    // per local device
    std::vector<uint32_t *> d_local;     // per local device: its local array (none for rank 0 in place)
    uint64_t nchecksums = 0;
    bool self_send = false;
    std::vector<Xfer> xfers;  // the gather's placements (group ranges), in posting order
    // packed gather: one send per sender of its whole local array into rank
    // 0's staging array (stage_off per rank), then the scatter kernel
    bool packed = false;
    std::vector<uint64_t> stage_off;  // per rank (senders only)
    uint64_t stage_n = 0;
    uint32_t *d_stage = nullptr;       // on rank 0's device
    ScatterTile *d_tiles = nullptr;    // on rank 0's device
    uint32_t ntiles = 0;
    int root_local = -1;  // local device index of rank 0 (-1: not in this process)
    // Successive execs reuse d_local (an exec's sends read it while the next
    // exec's kernel rewrites it): per local device, the stream of the
    // previous exec; an exec on another stream first waits for an event
    // recorded on that one at the switch (same stream: stream order, no call).
    std::vector<hipStream_t> last_stream;
    std::vector<hipEvent_t> last_done;
    std::vector<char> launched;
    // CRC32C_MULTI_PIPELINE: per local device, the plan's two exec streams
    // and events (Pipe), a second local array (exec k uses array k % 2),
    // the execs issued so far, the previous exec's root_out, and the gather
    // of the previous exec, issued by the next exec (or the join) on the
    // caller's streams -- after the next exec's fork point, so that exec's
    // launch runs beside this gather.
    bool pipeline = false;
    struct Pipe {
        hipStream_t exec[2] = {nullptr, nullptr};  // exec k's shard launch on exec[k % 2]
        hipEvent_t fork = nullptr;                 // on the caller's stream at an exec
        hipEvent_t kern[2] = {nullptr, nullptr};   // exec[b] after its launch
        hipEvent_t tail = nullptr;                 // crc32c_multi_plan_join
        uint64_t cap = 0;  // the caller's capture the streams follow (0: none; follow_capture)
        bool kern_rec[2] = {false, false};  // recorded, still to be waited on
        bool used[2] = {false, false};      // exec[b] issued since the last join
    };
    std::vector<Pipe> pipes;
    std::vector<uint32_t *> d_local2;  // per local device: local array 1
    uint64_t nexec = 0;
    uint32_t *last_root = nullptr;
    bool gather_pending = false;  // the previous exec's gather is not issued yet
    uint32_t pend_b = 0;          // ... its local arrays and root_out
    uint32_t *pend_root = nullptr;
};

namespace {

// Before an exec on `s` (local device i): when the previous exec of the plan
// went on another stream, an event recorded on that stream now (it follows
// everything issued there so far, the previous exec's sends included) is
// waited on -- by `s`, or by the host while `s` is being captured (a capture
// cannot wait on work outside it).  A previous exec captured into a graph
// needs nothing: its replays are ordered by the caller's graph launches.
int order_exec(crc32c_multi_plan *mp, size_t i, hipStream_t s) {
    if (!mp->launched[i] || mp->last_stream[i] == s) return 0;
    crc32c_multi *m = mp->m;
    DeviceGuard guard(m->ctxs[i]->device);
    hipStreamCaptureStatus prev = hipStreamCaptureStatusNone, cur = hipStreamCaptureStatusNone;
    HIP_TRY(hipStreamIsCapturing(mp->last_stream[i], &prev));
    if (prev != hipStreamCaptureStatusNone) return 0;
    HIP_TRY(hipEventRecord(mp->last_done[i], mp->last_stream[i]));
    HIP_TRY(hipStreamIsCapturing(s, &cur));
    if (cur != hipStreamCaptureStatusNone) {
        RelaxedCapture relaxed;  // (a host wait on this thread during its capture)
        HIP_TRY(hipEventSynchronize(mp->last_done[i]));
    } else {
        HIP_TRY(hipStreamWaitEvent(s, mp->last_done[i], 0));
    }
    return 0;
}

// 1 + the capture id of `s` (0: not capturing; HIP's ids may start at 0).
int capture_id(hipStream_t s, uint64_t *id) {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    unsigned long long cid = 0;
    HIP_TRY(hipStreamGetCaptureInfo(s, &st, &cid));
    *id = st == hipStreamCaptureStatusActive ? uint64_t(cid) + 1 : 0;
    return 0;
}

// The plan's exec streams of one local device follow the caller's stream
// `s` into (or out of) a graph capture.  Entering one: they are drained by
// the host first (they hold only work from before the capture), so no wait
// inside the capture names an event recorded outside it (HIP refuses a host
// wait on an event whose stream has since joined a capture, and a capture
// cannot wait on work outside it).  Leaving one: the events recorded inside
// it are graph nodes, ordered by the caller's graph launches.  Either way
// the pending waits are dropped.
int follow_capture(crc32c_multi_plan::Pipe &P, hipStream_t s) {
    uint64_t cur = 0;
    if (int rc = capture_id(s, &cur)) return rc;
    if (cur == P.cap) return 0;
    if (P.cap == 0) {
        RelaxedCapture relaxed;  // (host waits on this thread during its capture)
        for (hipStream_t x : P.exec) HIP_TRY(hipStreamSynchronize(x));
    }
    P.cap = cur;
    P.kern_rec[0] = P.kern_rec[1] = false;
    return 0;
}

// One RCCL group of the gather, from every local device's local array
// (src[i]) into root_out, on its stream -- per placement, or packed (one
// operation per sender into the staging array) -- then, packed, the scatter
// kernel on rank 0's stream.
int post_gather(crc32c_multi_plan *mp, const std::vector<const uint32_t *> &src, uint32_t *root_out,
                void *const *streams) {
    crc32c_multi *m = mp->m;
    NCCL_TRY(rccl().GroupStart());
    ncclResult_t r = ncclSuccess;
    for (size_t i = 0; i < m->ctxs.size() && r == ncclSuccess; ++i) {
        const hipStream_t s = local_stream(m, i, streams);
        const int me = m->ranks[i];
        if (mp->packed) {
            if (sends(me, mp->self_send) && mp->local_nout[size_t(me)])
                r = rccl().Send(src[i], mp->local_nout[size_t(me)], ncclUint32, 0, m->comms[i], s);
            for (int q = 0; me == 0 && q < m->nranks && r == ncclSuccess; ++q)
                if (sends(q, mp->self_send) && mp->local_nout[size_t(q)])
                    r = rccl().Recv(mp->d_stage + mp->stage_off[size_t(q)], mp->local_nout[size_t(q)], ncclUint32, q,
                                    m->comms[i], s);
            continue;
        }
        for (const Xfer &x : mp->xfers) {
            if (r != ncclSuccess) break;
            if (x.rank == me) r = rccl().Send(src[i] + x.local, x.count, ncclUint32, 0, m->comms[i], s);
            if (me == 0 && r == ncclSuccess) r = rccl().Recv(root_out + x.file, x.count, ncclUint32, x.rank, m->comms[i], s);
        }
    }
    const ncclResult_t e = rccl().GroupEnd();
    NCCL_TRY(r);
    NCCL_TRY(e);
    if (mp->packed && mp->root_local >= 0 && mp->ntiles) {
        const size_t i = size_t(mp->root_local);
        DeviceGuard guard(m->ctxs[i]->device);
        hipLaunchKernelGGL(hdfs_crc32c_gather_scatter, dim3(mp->ntiles), dim3(256), 0, local_stream(m, i, streams),
                           mp->d_stage, root_out, mp->d_tiles);
        HIP_TRY(hipGetLastError());
    }
    return 0;
}

// The gather of the exec that used local arrays b, into root_out: on every
// local device's caller stream, after that exec's launch (an event wait),
// one RCCL group (the same transfers as an ordinary exec's).
int issue_gather(crc32c_multi_plan *mp, uint32_t b, uint32_t *root_out, void *const *streams) {
    crc32c_multi *m = mp->m;
    if (int rc = ensure_comms(m)) return rc;
    for (size_t i = 0; i < m->ctxs.size(); ++i) {
        crc32c_multi_plan::Pipe &P = mp->pipes[i];
        DeviceGuard guard(m->ctxs[i]->device);
        const hipStream_t s = local_stream(m, i, streams);
        if (int rc = follow_capture(P, s)) return rc;
        if (P.kern_rec[b]) HIP_TRY(hipStreamWaitEvent(s, P.kern[b], 0));
    }
    std::vector<const uint32_t *> src(m->ctxs.size());
    for (size_t i = 0; i < m->ctxs.size(); ++i) src[i] = b ? mp->d_local2[i] : mp->d_local[i];
    return post_gather(mp, src, root_out, streams);
}

// One pipelined exec (CRC32C_MULTI_PIPELINE; see crc32c_multi_plan_exec).
int exec_pipelined(crc32c_multi_plan *mp, const void *const *dev_shards, uint32_t *root_out, void *const *streams) {
    crc32c_multi *m = mp->m;
    const uint32_t b = uint32_t(mp->nexec & 1u);
    const bool same_root = root_out && root_out == mp->last_root;
    // 1. every local device's shard launch on the plan's exec stream b,
    //    forked from the caller's stream: after the caller's work so far --
    //    the gather of exec k - 2, the last reader of local array b,
    //    included -- but not after exec k - 1's launch (on exec[1 - b]) or
    //    gather (issued below); after exec k - 1's launch only when both
    //    write the same root_out in place
    for (size_t i = 0; i < m->ctxs.size(); ++i) {
        crc32c_multi_plan::Pipe &P = mp->pipes[i];
        DeviceGuard guard(m->ctxs[i]->device);
        const hipStream_t s = local_stream(m, i, streams), E = P.exec[b];
        if (int rc = follow_capture(P, s)) return rc;
        HIP_TRY(hipEventRecord(P.fork, s));
        HIP_TRY(hipStreamWaitEvent(E, P.fork, 0));
        P.used[b] = true;
        if (!mp->local_nout[size_t(m->ranks[i])]) continue;
        const bool in_place = !mp->d_local[i];
        if (in_place && same_root && P.kern_rec[1 - b]) HIP_TRY(hipStreamWaitEvent(E, P.kern[1 - b], 0));
        uint32_t *dst = in_place ? root_out : (b ? mp->d_local2[i] : mp->d_local[i]);
        if (int rc = crc32c_plan_exec(mp->plans[i], dev_shards[i], dst, E)) return rc;
        HIP_TRY(hipEventRecord(P.kern[b], E));
        P.kern_rec[b] = true;
    }
    mp->last_root = root_out;
    mp->nexec++;
    // 2. exec k - 1's gather, now (it runs beside this launch); this exec's
    //    waits for the next exec or the join
    if (mp->gather_pending) {
        mp->gather_pending = false;
        if (int rc = issue_gather(mp, mp->pend_b, mp->pend_root, streams)) return rc;
    }
    if (!mp->xfers.empty()) {
        mp->gather_pending = true;
        mp->pend_b = b;
        mp->pend_root = root_out;
    }
    return 0;
}

}  // namespace

extern "C" {

int crc32c_multi_create(const int *devices, int ndevices, crc32c_multi **out) {
    if (!out || ndevices <= 0) return fail(-EINVAL, "bad arguments");
    *out = nullptr;
    std::unique_ptr<crc32c_multi, int (*)(crc32c_multi *)> m(new crc32c_multi, crc32c_multi_destroy);
    m->nranks = ndevices;
    for (int i = 0; i < ndevices; ++i) {
        crc32c_ctx *c = nullptr;
        if (int rc = crc32c_ctx_create(devices ? devices[i] : i, &c)) return rc;
        m->ctxs.push_back(c);
        m->ranks.push_back(i);
        hipStream_t s = nullptr;
        DeviceGuard guard(c->device);
        HIP_TRY(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        m->streams.push_back(s);
    }
    *out = m.release();
    return 0;
}

int crc32c_multi_unique_id(uint8_t id[128]) {
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId is 128 bytes");
    if (!id) return fail(-EINVAL, "id == NULL");
    ncclUniqueId u;
    RCCL_LOADED();
    NCCL_TRY(rccl().GetUniqueId(&u));
    std::memcpy(id, &u, sizeof u);
    return 0;
}

int crc32c_multi_create_rank(int device, int rank, int nranks, const uint8_t id[128], crc32c_multi **out) {
    if (!out || !id || nranks <= 0 || rank < 0 || rank >= nranks) return fail(-EINVAL, "bad arguments");
    *out = nullptr;
    std::unique_ptr<crc32c_multi, int (*)(crc32c_multi *)> m(new crc32c_multi, crc32c_multi_destroy);
    m->nranks = nranks;
    crc32c_ctx *c = nullptr;
    if (int rc = crc32c_ctx_create(device, &c)) return rc;
    m->ctxs.push_back(c);
    m->ranks.push_back(rank);
    DeviceGuard guard(device);
    hipStream_t s = nullptr;
    HIP_TRY(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    m->streams.push_back(s);
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof u);
    ncclComm_t comm = nullptr;
    RCCL_LOADED();
    NCCL_TRY(rccl().CommInitRank(&comm, nranks, u, rank));
    m->comms.push_back(comm);
    *out = m.release();
    return 0;
}

int crc32c_multi_destroy(crc32c_multi *m) {
    if (!m) return 0;
    for (size_t i = 0; i < m->ctxs.size(); ++i) {
        DeviceGuard guard(m->ctxs[i]->device);
        if (i < m->streams.size() && m->streams[i]) {
            (void)hipStreamSynchronize(m->streams[i]);
            (void)hipStreamDestroy(m->streams[i]);
        }
        if (i < m->comms.size() && m->comms[i]) (void)rccl().CommDestroy(m->comms[i]);
    }
    for (crc32c_ctx *c : m->ctxs) crc32c_ctx_destroy(c);
    delete m;
    return 0;
}

int crc32c_multi_sync(crc32c_multi *m) {
    if (!m) return fail(-EINVAL, "multi == NULL");
    for (size_t i = 0; i < m->ctxs.size(); ++i) {
        DeviceGuard guard(m->ctxs[i]->device);
        HIP_TRY(hipStreamSynchronize(m->streams[i]));
    }
    return 0;
}

int64_t crc32c_multi_layout(const crc32c_packet *pkts, size_t npkts, uint32_t group_packets, int nranks,
                            uint64_t *layout, uint64_t *shard_bytes) {
    std::vector<Group> groups;
    std::vector<uint64_t> sb, ln;
    if (int rc = build_layout(pkts, npkts, group_packets, nranks, &groups, &sb, &ln)) return rc;
    for (size_t g = 0; layout && g < groups.size(); ++g) {
        layout[4 * g] = uint64_t(groups[g].rank);
        layout[4 * g + 1] = groups[g].shard_off;
        layout[4 * g + 2] = groups[g].lo;
        layout[4 * g + 3] = groups[g].hi - groups[g].lo;
    }
    if (shard_bytes) std::copy(sb.begin(), sb.end(), shard_bytes);
    return int64_t(groups.size());
}

int64_t crc32c_multi_shard_packets(const crc32c_packet *pkts, size_t npkts, uint32_t group_packets, int nranks,
                                   int rank, crc32c_packet *local, size_t cap) {
    std::vector<Group> groups;
    std::vector<uint64_t> sb, ln;
    if (int rc = build_layout(pkts, npkts, group_packets, nranks, &groups, &sb, &ln)) return rc;
    if (rank < 0 || rank >= nranks) return fail(-EINVAL, "rank %d out of range", rank);
    std::vector<crc32c_packet> v;
    shard_packets(pkts, npkts, group_packets, groups, rank, false, &v);
    if (local) std::copy(v.begin(), v.begin() + std::min(cap, v.size()), local);
    return int64_t(v.size());
}

int64_t crc32c_multi_rank_packets(const crc32c_packet *pkts, size_t npkts, uint32_t group_packets, int nranks,
                                  int rank, uint32_t flags, crc32c_packet *local, size_t cap) {
    std::vector<Group> groups;
    std::vector<uint64_t> sb, ln;
    if (int rc = build_layout(pkts, npkts, group_packets, nranks, &groups, &sb, &ln)) return rc;
    if (rank < 0 || rank >= nranks) return fail(-EINVAL, "rank %d out of range", rank);
    std::vector<crc32c_packet> v;
    rank_plan_packets(pkts, npkts, group_packets, groups, rank, (flags & CRC32C_MULTI_SELF_SEND) != 0, &v);
    if (local) std::copy(v.begin(), v.begin() + std::min(cap, v.size()), local);
    return int64_t(v.size());
}

int64_t crc32c_multi_transfers(const crc32c_packet *pkts, size_t npkts, uint32_t group_packets, int nranks,
                               uint32_t flags, uint64_t *local_nout, uint64_t *xfers, size_t cap) {
    std::vector<Group> groups;
    std::vector<uint64_t> sb, ln;
    if (int rc = build_layout(pkts, npkts, group_packets, nranks, &groups, &sb, &ln)) return rc;
    const bool self_send = (flags & CRC32C_MULTI_SELF_SEND) != 0;
    std::vector<Xfer> xs;
    build_transfers(groups, self_send, &xs);
    for (int r = 0; local_nout && r < nranks; ++r) local_nout[r] = sends(r, self_send) ? ln[size_t(r)] : 0;
    for (size_t k = 0; xfers && k < std::min(cap, xs.size()); ++k) {
        xfers[4 * k] = uint64_t(xs[k].rank);
        xfers[4 * k + 1] = xs[k].local;
        xfers[4 * k + 2] = xs[k].file;
        xfers[4 * k + 3] = xs[k].count;
    }
    return int64_t(xs.size());
}

int64_t crc32c_multi_scatter(const crc32c_packet *pkts, size_t npkts, uint32_t group_packets, int nranks,
                             uint32_t flags, uint64_t *stage_off, uint64_t *tiles, size_t cap) {
    std::vector<Group> groups;
    std::vector<uint64_t> sb, ln;
    if (int rc = build_layout(pkts, npkts, group_packets, nranks, &groups, &sb, &ln)) return rc;
    const bool self_send = (flags & CRC32C_MULTI_SELF_SEND) != 0;
    std::vector<Xfer> xs;
    build_transfers(groups, self_send, &xs);
    for (int r = 0; stage_off && r < nranks; ++r) stage_off[r] = 0;
    if ((flags & CRC32C_MULTI_PER_GROUP_RECV) || !wants_packed(xs)) return 0;
    std::vector<uint64_t> so;
    stage_offsets(ln, self_send, &so);
    if (stage_off) std::copy(so.begin(), so.end(), stage_off);
    std::vector<ScatterTile> ts;
    build_scatter(xs, so, &ts);
    for (size_t k = 0; tiles && k < std::min(cap, ts.size()); ++k) {
        tiles[3 * k] = ts[k].src;
        tiles[3 * k + 1] = ts[k].dst;
        tiles[3 * k + 2] = ts[k].n;
    }
    return int64_t(ts.size());
}

int crc32c_multi_plan_create(crc32c_multi *m, const crc32c_packet *pkts, size_t npkts, uint32_t group_packets,
                             uint32_t flags, crc32c_multi_plan **out) {
    if (!m || !out) return fail(-EINVAL, "multi/out == NULL");
    *out = nullptr;
    if (flags & (CRC32C_DEVICE_ADDRESSES | CRC32C_CPU_FALLBACK))
        return fail(-EINVAL, "flags 0x%x not valid for a multi-GPU plan", flags);
    if (group_packets == 0) group_packets = 64;
    // RCCL has one rank per GPU: a one-process communicator (ncclCommInitAll)
    // cannot list a device twice (crc32c_multi_batch_host can: it uses no RCCL)
    for (size_t i = 0; i < m->ctxs.size(); ++i)
        for (size_t j = 0; j < i; ++j)
            if (m->ctxs[i]->device == m->ctxs[j]->device)
                return fail(-EINVAL, "device %d is listed twice: a multi-GPU plan needs one rank per GPU",
                            m->ctxs[i]->device);
    std::unique_ptr<crc32c_multi_plan, int (*)(crc32c_multi_plan *)> mp(new crc32c_multi_plan,
                                                                        crc32c_multi_plan_destroy);
    mp->m = m;
    mp->last_stream.assign(m->ctxs.size(), nullptr);
    mp->last_done.assign(m->ctxs.size(), nullptr);
    mp->launched.assign(m->ctxs.size(), 0);
    for (size_t i = 0; i < m->ctxs.size(); ++i) {
        DeviceGuard guard(m->ctxs[i]->device);
        HIP_TRY(hipEventCreateWithFlags(&mp->last_done[i], hipEventDisableTiming));
    }
    mp->self_send = (flags & CRC32C_MULTI_SELF_SEND) != 0;
    mp->pipeline = (flags & CRC32C_MULTI_PIPELINE) != 0;
    const bool per_group = (flags & CRC32C_MULTI_PER_GROUP_RECV) != 0;
    flags &= ~(CRC32C_MULTI_SELF_SEND | CRC32C_MULTI_PIPELINE | CRC32C_MULTI_PER_GROUP_RECV);
    if (int rc = build_layout(pkts, npkts, group_packets, m->nranks, &mp->groups, &mp->shard_bytes, &mp->local_nout))
        return rc;
    for (const Group &G : mp->groups) mp->nchecksums = std::max(mp->nchecksums, G.omin + G.n);
    std::vector<crc32c_packet> local;
    for (size_t i = 0; i < m->ctxs.size(); ++i) {
        const int r = m->ranks[i];
        // rank 0 in place: its packets keep their global out indices
        const bool in_place = !sends(r, mp->self_send);
        if (r == 0) mp->root_local = int(i);
        rank_plan_packets(pkts, npkts, group_packets, mp->groups, r, mp->self_send, &local);
        crc32c_plan *p = nullptr;
        if (int rc = crc32c_plan_create(m->ctxs[i], local.data(), local.size(), flags, &p)) return rc;
        mp->plans.push_back(p);
        uint32_t *d = nullptr;
        if (!in_place && mp->local_nout[size_t(r)]) {
            DeviceGuard guard(m->ctxs[i]->device);
            HIP_TRY(hipMalloc(reinterpret_cast<void **>(&d), mp->local_nout[size_t(r)] * sizeof(uint32_t)));
        }
        mp->d_local.push_back(d);
        uint32_t *d2 = nullptr;
        if (mp->pipeline && d) {
            DeviceGuard guard(m->ctxs[i]->device);
            HIP_TRY(hipMalloc(reinterpret_cast<void **>(&d2), mp->local_nout[size_t(r)] * sizeof(uint32_t)));
        }
        mp->d_local2.push_back(d2);
    }
    if (mp->pipeline) {
        mp->pipes.resize(m->ctxs.size());
        for (size_t i = 0; i < m->ctxs.size(); ++i) {
            crc32c_multi_plan::Pipe &P = mp->pipes[i];
            DeviceGuard guard(m->ctxs[i]->device);
            for (hipStream_t *st : {&P.exec[0], &P.exec[1]}) HIP_TRY(hipStreamCreateWithFlags(st, hipStreamNonBlocking));
            for (hipEvent_t *ev : {&P.fork, &P.kern[0], &P.kern[1], &P.tail})
                HIP_TRY(hipEventCreateWithFlags(ev, hipEventDisableTiming));
        }
    }
    build_transfers(mp->groups, mp->self_send, &mp->xfers);
    if (mp->nchecksums > UINT32_MAX) return fail(-E2BIG, "too many checksums");
    mp->packed = !per_group && wants_packed(mp->xfers);
    // (per placement, every transfer is one ncclSend / ncclRecv of the exec's
    // one RCCL group: bounded, so a tiny group_packets cannot post thousands
    // of point-to-point operations per exec)
    if (!mp->packed && mp->xfers.size() > kMaxGatherTransfers)
        return fail(-E2BIG, "%zu gather transfers (at most %zu): use a larger group_packets", mp->xfers.size(),
                    kMaxGatherTransfers);
    if (mp->packed) {
        mp->stage_n = stage_offsets(mp->local_nout, mp->self_send, &mp->stage_off);
        if (mp->root_local >= 0) {
            std::vector<ScatterTile> tiles;
            build_scatter(mp->xfers, mp->stage_off, &tiles);
            if (tiles.size() > 0x7fffffffu) return fail(-E2BIG, "too many scatter tiles");
            mp->ntiles = uint32_t(tiles.size());
            DeviceGuard guard(m->ctxs[size_t(mp->root_local)]->device);
            HIP_TRY(hipMalloc(reinterpret_cast<void **>(&mp->d_stage), std::max<uint64_t>(mp->stage_n, 1) * 4));
            HIP_TRY(hipMalloc(reinterpret_cast<void **>(&mp->d_tiles),
                              std::max<size_t>(tiles.size(), 1) * sizeof(ScatterTile)));
            HIP_TRY(hipMemcpy(mp->d_tiles, tiles.data(), tiles.size() * sizeof(ScatterTile), hipMemcpyHostToDevice));
        }
    }
    *out = mp.release();
    return 0;
}

uint64_t crc32c_multi_plan_gather_ops(const crc32c_multi_plan *mp, int *packed) {
    if (packed) *packed = mp ? int(mp->packed) : 0;
    if (!mp) return 0;
    if (!mp->packed) return 2 * uint64_t(mp->xfers.size());
    uint64_t senders = 0;
    for (int q = 0; q < mp->m->nranks; ++q) senders += sends(q, mp->self_send) && mp->local_nout[size_t(q)] ? 1 : 0;
    return 2 * senders;
}

uint64_t crc32c_multi_plan_nchecksums(const crc32c_multi_plan *mp) { return mp ? mp->nchecksums : 0; }

uint64_t crc32c_multi_plan_shard_bytes(const crc32c_multi_plan *mp, int rank) {
    if (!mp || rank < 0 || size_t(rank) >= mp->shard_bytes.size()) return 0;
    return mp->shard_bytes[size_t(rank)];
}

int crc32c_multi_plan_exec(crc32c_multi_plan *mp, const void *const *dev_shards, uint32_t *root_out,
                           void *const *streams) {
    if (!mp) return fail(-EINVAL, "plan == NULL");
    crc32c_multi *m = mp->m;
    std::lock_guard<std::mutex> lock(m->mu);
    for (size_t i = 0; i < m->ctxs.size(); ++i)
        if (mp->local_nout[size_t(m->ranks[i])] && (!dev_shards || !dev_shards[i]))
            return fail(-EINVAL, "local device %zu: shard payload == NULL", i);
    if (mp->root_local >= 0 && mp->nchecksums && !root_out) return fail(-EINVAL, "root_out == NULL on rank 0");
    if (mp->pipeline) return exec_pipelined(mp, dev_shards, root_out, streams);
    // 0. after the previous exec when it ran on another stream (its sends may
    //    still read the local arrays this one overwrites)
    for (size_t i = 0; i < m->ctxs.size(); ++i)
        if (int rc = order_exec(mp, i, local_stream(m, i, streams))) return rc;
    for (size_t i = 0; i < m->ctxs.size(); ++i) {
        mp->last_stream[i] = local_stream(m, i, streams);
        mp->launched[i] = 1;
    }
    // 1. every local device checksums its shard: rank 0 into place, the
    //    others into their local arrays
    for (size_t i = 0; i < m->ctxs.size(); ++i) {
        if (!mp->local_nout[size_t(m->ranks[i])]) continue;
        uint32_t *dst = mp->d_local[i] ? mp->d_local[i] : root_out;
        if (int rc = crc32c_plan_exec(mp->plans[i], dev_shards[i], dst, local_stream(m, i, streams))) return rc;
    }
    // 2. one group of point-to-point transfers: every sender's group ranges
    //    from its local array, rank 0's receives straight into file order
    if (mp->xfers.empty()) return 0;
    if (int rc = ensure_comms(m)) return rc;
    std::vector<const uint32_t *> src(mp->d_local.begin(), mp->d_local.end());
    return post_gather(mp, src, root_out, streams);
}

int crc32c_multi_plan_join(crc32c_multi_plan *mp, void *const *streams) {
    if (!mp) return fail(-EINVAL, "plan == NULL");
    if (!mp->pipeline) return 0;  // (an ordinary exec is complete with its stream)
    crc32c_multi *m = mp->m;
    std::lock_guard<std::mutex> lock(m->mu);
    // the last exec's gather, then every exec stream's launches
    if (mp->gather_pending) {
        mp->gather_pending = false;
        if (int rc = issue_gather(mp, mp->pend_b, mp->pend_root, streams)) return rc;
    }
    for (size_t i = 0; i < m->ctxs.size(); ++i) {
        crc32c_multi_plan::Pipe &P = mp->pipes[i];
        DeviceGuard guard(m->ctxs[i]->device);
        const hipStream_t s = local_stream(m, i, streams);
        if (int rc = follow_capture(P, s)) return rc;
        for (int k = 0; k < 2; ++k) {
            if (!P.used[k]) continue;
            HIP_TRY(hipEventRecord(P.tail, P.exec[k]));
            HIP_TRY(hipStreamWaitEvent(s, P.tail, 0));
            P.used[k] = false;
        }
    }
    return 0;
}

int crc32c_multi_plan_destroy(crc32c_multi_plan *mp) {
    if (!mp) return 0;
    // (the plan's own streams drain first; the shard plans then need no
    // event on them at their release)
    for (size_t i = 0; i < mp->pipes.size(); ++i) {
        crc32c_multi_plan::Pipe &P = mp->pipes[i];
        DeviceGuard guard(mp->m->ctxs[i]->device);
        for (hipStream_t st : P.exec)
            if (st) {
                (void)hipStreamSynchronize(st);
                if (i < mp->plans.size()) plan_forget_stream(mp->plans[i], st);
            }
    }
    for (size_t i = 0; i < mp->last_done.size(); ++i)
        if (mp->last_done[i]) {
            DeviceGuard guard(mp->m->ctxs[i]->device);
            (void)hipEventDestroy(mp->last_done[i]);
        }
    for (size_t i = 0; i < mp->plans.size(); ++i) {
        crc32c_plan_destroy(mp->plans[i]);
        DeviceGuard guard(mp->m->ctxs[i]->device);
        if (i < mp->d_local.size() && mp->d_local[i]) (void)hipFree(mp->d_local[i]);
        if (i < mp->d_local2.size() && mp->d_local2[i]) (void)hipFree(mp->d_local2[i]);
    }
    if (mp->root_local >= 0 && (mp->d_stage || mp->d_tiles)) {
        DeviceGuard guard(mp->m->ctxs[size_t(mp->root_local)]->device);
        if (mp->d_stage) (void)hipFree(mp->d_stage);
        if (mp->d_tiles) (void)hipFree(mp->d_tiles);
    }
    for (size_t i = 0; i < mp->pipes.size(); ++i) {
        crc32c_multi_plan::Pipe &P = mp->pipes[i];
        DeviceGuard guard(mp->m->ctxs[i]->device);
        for (hipStream_t st : P.exec)
            if (st) (void)hipStreamDestroy(st);
        for (hipEvent_t ev : {P.fork, P.kern[0], P.kern[1], P.tail})
            if (ev) (void)hipEventDestroy(ev);
    }
    delete mp;
    return 0;
}

int crc32c_multi_batch_host(crc32c_multi *m, const void *payload, const crc32c_packet *pkts, size_t npkts,
                            uint32_t group_packets, uint32_t *out, uint32_t flags) {
    if (!m || m->ctxs.empty()) return fail(-EINVAL, "multi == NULL");
    for (size_t i = 0; i < npkts; ++i)
        if (!pkts || (pkts[i].len && pkts[i].bpc == 0))
            return fail(-EINVAL, "packet %zu: bytesPerChecksum == 0", i);
    if (group_packets == 0) group_packets = 64;
    const size_t g = m->ctxs.size();
    // Groups of consecutive packets (an HDFS block's worth) dealt round-robin
    // over the local devices, each over its own PCIe link.
    std::vector<std::vector<crc32c_packet>> shard(g);
    for (size_t i = 0; i < npkts; ++i) shard[(i / group_packets) % g].push_back(pkts[i]);
    std::vector<int> rcs(g, 0);
    std::vector<std::string> errs(g);
    std::vector<std::thread> th;
    for (size_t d = 0; d < g; ++d)
        th.emplace_back([&, d] {
            rcs[d] = crc32c_batch_host(m->ctxs[d], payload, shard[d].data(), shard[d].size(), out,
                                       flags & ~CRC32C_CPU_FALLBACK);
            if (rcs[d]) errs[d] = crc32c_last_error();
        });
    for (auto &t : th) t.join();
    for (size_t d = 0; d < g; ++d)
        if (rcs[d]) return fail(rcs[d], "device %d: %s", m->ctxs[d]->device, errs[d].c_str());
    return 0;
}

}  // extern "C"
