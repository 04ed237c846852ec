// errors.h -- the library's error reporting (not part of the C ABI): every
// entry point that fails sets the calling thread's crc32c_last_error() text
// through fail() and returns its code (0 / -errno, the reference's
// convention, src/hadooprpc.c:440-486).
#pragma once

namespace hdfs_crc {

// Sets the calling thread's error text; returns `code`.
int fail(int code, const char *fmt, ...) __attribute__((format(printf, 2, 3)));

}  // namespace hdfs_crc
