# What HIP returns for calls on a stream the caller has already destroyed.
import ctypes, sys
hip = ctypes.CDLL("libamdhip64.so")
def rc(name, *a):
    r = getattr(hip, name)(*a)
    print(name, r, flush=True)
    return r
s = ctypes.c_void_p()
rc("hipSetDevice", 0)
rc("hipStreamCreate", ctypes.byref(s))
rc("hipStreamDestroy", s)
st = ctypes.c_int(0)
rc("hipStreamQuery", s)
rc("hipStreamIsCapturing", s, ctypes.byref(st))
e = ctypes.c_void_p()
rc("hipEventCreateWithFlags", ctypes.byref(e), 2)
rc("hipEventRecord", e, s)
rc("hipEventQuery", e)
s2 = ctypes.c_void_p()
rc("hipStreamCreate", ctypes.byref(s2))
print("reused handle", s.value == s2.value, flush=True)
print("probe done", flush=True)
