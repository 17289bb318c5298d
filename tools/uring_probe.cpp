// tools/uring_probe.cpp — is io_uring usable here (seccomp / sysctl)? Sets up a ring and reports the
// kernel's feature bits and whether the opcodes the loader would use are supported.
// Build: g++ -O2 tools/uring_probe.cpp -o build/bin/uring_probe
#include <linux/io_uring.h>
#include <sys/syscall.h>
#include <unistd.h>
#include <cerrno>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <sys/mman.h>
int main() {
  io_uring_params p;
  std::memset(&p, 0, sizeof(p));
  const int fd = (int)syscall(SYS_io_uring_setup, 64, &p);
  if (fd < 0) {
    std::printf("io_uring_setup failed: %s\n", std::strerror(errno));
    return 0;
  }
  std::printf("io_uring ok: features 0x%x sq %u cq %u\n", p.features, p.sq_entries, p.cq_entries);
  const size_t sz = sizeof(io_uring_probe) + 256 * sizeof(io_uring_probe_op);
  auto* pr = (io_uring_probe*)std::calloc(1, sz);
  if (syscall(SYS_io_uring_register, fd, IORING_REGISTER_PROBE, pr, 256) == 0) {
    const int ops[] = {IORING_OP_OPENAT, IORING_OP_READ, IORING_OP_CLOSE, IORING_OP_WRITEV, IORING_OP_WRITE, IORING_OP_STATX};
    const char* nm[] = {"OPENAT", "READ", "CLOSE", "WRITEV", "WRITE", "STATX"};
    for (int i = 0; i < 6; ++i)
      std::printf("  %s %s\n", nm[i], ops[i] <= pr->last_op && (pr->ops[ops[i]].flags & IO_URING_OP_SUPPORTED) ? "yes" : "no");
  } else {
    std::printf("probe failed: %s\n", std::strerror(errno));
  }
  close(fd);
  return 0;
}
