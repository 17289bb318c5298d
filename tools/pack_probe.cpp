// tools/pack_probe.cpp — per-slice host costs of the loader pieces on one thread: 12-bit pack of a
// 256² slice into pinned-like memory (streaming stores), open + pread + close of a 131 KB tmpfs file,
// a 131 KB memcpy. Build: g++ -O2 -Iinclude tools/pack_probe.cpp -Lnm03_capstone_project_amd/lib -lnm03
//   -Wl,-rpath,$PWD/nm03_capstone_project_amd/lib -o build/bin/pack_probe
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cstring>
#include <fcntl.h>
#include <unistd.h>
#include "nm03/pack12.h"
#ifndef NSLOT
#define NSLOT 300
#endif
int main() {
  const size_t n = 65536;
  std::vector<uint16_t> src(n);
  for (size_t i = 0; i < n; ++i) src[i] = (uint16_t)((i * 2654435761u) & 0xFFF);
  std::vector<uint8_t> dst(64 << 20);
  const int reps = 2000;
  auto t0 = std::chrono::steady_clock::now();
  for (int r = 0; r < reps; ++r) nm03::pack12::pack_stream(src.data(), n, dst.data() + (size_t)(r % NSLOT) * 98304);
  auto t1 = std::chrono::steady_clock::now();
  for (int r = 0; r < reps; ++r) nm03::pack12::pack_stream_checked(src.data(), n, dst.data() + (size_t)(r % NSLOT) * 98304);
  auto t2 = std::chrono::steady_clock::now();
  // pread from tmpfs file
  const char* p = "/dev/shm/pb_test.bin";
  int fd = open(p, O_CREAT | O_RDWR | O_TRUNC, 0644); std::vector<uint8_t> f(131*1024, 3); if (write(fd, f.data(), f.size()) < 0) return 1; close(fd);
  std::vector<uint8_t> buf(256 * 1024);
  auto t3 = std::chrono::steady_clock::now();
  for (int r = 0; r < reps; ++r) { int fd2 = open(p, O_RDONLY); if (pread(fd2, buf.data(), 256*1024, 0) < 0) return 1; close(fd2); }
  auto t4 = std::chrono::steady_clock::now();
  for (int r = 0; r < reps; ++r) { memcpy(buf.data(), dst.data() + (size_t)(r % 300) * 131072 % (60<<20), 131*1024); }
  auto t5 = std::chrono::steady_clock::now();
  unlink(p);
  auto us = [&](auto a, auto b) { return std::chrono::duration<double>(b - a).count() * 1e6 / reps; };
  printf("pack_stream %.2f us, checked %.2f us, open+pread+close(131KB tmpfs, cache-hot) %.2f us, memcpy 131KB %.2f us\n", us(t0, t1), us(t1, t2), us(t3, t4), us(t4,t5));
}
