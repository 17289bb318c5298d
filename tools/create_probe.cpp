// tools/create_probe.cpp — what does creating and deleting a small output file cost on this host,
// and is it contention or a floor?
// Build: g++ -O2 -pthread tools/create_probe.cpp -o build/bin/create_probe
//
//   create_probe <root> <threads,...> <slices> <reps>
//
// Every worker runs like an engine pool worker (private fd table + private struct cred). A "slice"
// is two ≈12 KB JPEG-sized files. For each thread count and directory layout it times, per rep:
//   write   : each slice's two files created (O_CREAT|O_EXCL) + pwritev + close   [cold export]
//   tmpfile : O_TMPFILE in the directory + pwritev + linkat to its name + close       [cold export]
//   rewrite : the same files opened without O_CREAT + pwritev + close                 [warm export]
//   wipe    : every file unlinked (workers take whole directories, as setup_output_dirs does)
//   rename  : each directory renamed into a trash directory and re-created (the wipe's critical-path
//             part when a reaper deletes the trash later); the trash is then unlinked (reap)
// Layouts: shared  = slices dealt round-robin over 20 patient dirs, worker t takes slices t, t+T, ...
//                    (the engine's interleaved export order);
//          affine  = worker t writes only into dirs d ≡ t (mod T) (directory-affine writers);
//          private = one directory per worker.
// Output: CPU µs per slice (thread CPU clocks summed over workers) and the wall time per phase.
#include <dirent.h>
#include <fcntl.h>
#include <linux/capability.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <sys/uio.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <thread>
#include <vector>

#ifndef O_TMPFILE
#define O_TMPFILE (020000000 | O_DIRECTORY)
#endif
#ifndef CLOSE_RANGE_UNSHARE
#define CLOSE_RANGE_UNSHARE (1U << 1)
#endif

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
static long long tcpu() {
  timespec t;
  clock_gettime(CLOCK_THREAD_CPUTIME_ID, &t);
  return t.tv_sec * 1000000000LL + t.tv_nsec;
}
static void private_worker() {
  if (syscall(SYS_close_range, 3u, ~0u, CLOSE_RANGE_UNSHARE) != 0) perror("close_range");
  __user_cap_header_struct h{_LINUX_CAPABILITY_VERSION_3, 0};
  __user_cap_data_struct c[2]{};
  if (syscall(SYS_capget, &h, c) == 0) (void)syscall(SYS_capset, &h, c);
}

struct Phase {
  std::atomic<long long> cpu{0};
  double wall = 0;
};

// Runs fn(t) on T fresh private workers; returns summed thread CPU (ns) and wall.
static void run(int T, Phase& ph, const std::function<void(int)>& fn) {
  ph.cpu = 0;
  std::atomic<int> ready{0};
  std::atomic<bool> go{false};
  std::vector<std::thread> th;
  for (int t = 0; t < T; ++t)
    th.emplace_back([&, t] {
      private_worker();
      ready++;
      while (!go.load()) {
      }
      long long c0 = tcpu();
      fn(t);
      ph.cpu += tcpu() - c0;
    });
  while (ready.load() < T) {
  }
  double t0 = now();
  go = true;
  for (auto& x : th) x.join();
  ph.wall = now() - t0;
}

static void write_all(int fd, const uint8_t* p, size_t n) {
  iovec v{(void*)p, n};
  if (pwritev(fd, &v, 1, 0) != (ssize_t)n) {
    perror("pwritev");
    abort();
  }
}

int main(int argc, char** argv) {
  if (argc < 5) {
    fprintf(stderr, "usage: create_probe root threads[,threads...] slices reps\n");
    return 2;
  }
  const std::string root = argv[1];
  std::vector<int> Ts;
  for (char* s = argv[2]; *s;) {
    Ts.push_back((int)strtol(s, &s, 10));
    if (*s == ',') ++s;
  }
  const int nslices = atoi(argv[3]), reps = atoi(argv[4]);
  const size_t seg = 12000;
  std::vector<uint8_t> src((size_t)nslices * 2 * seg);
  for (size_t i = 0; i < src.size(); ++i) src[i] = (uint8_t)(i * 131);
  mkdir(root.c_str(), 0755);
  const std::string trash = root + "/.trash";
  mkdir(trash.c_str(), 0755);

  // Probe whether linkat(AT_EMPTY_PATH) works for our O_TMPFILE files (kernel >= 6.10 for non-root).
  std::atomic<int> empty_path_ok{-1};

  for (int T : Ts)
    for (int layout = 0; layout < 3; ++layout) {
      const char* lname = layout == 0 ? "shared" : layout == 1 ? "affine" : "private";
      const int nd = layout == 2 ? T : 20;
      std::vector<std::string> dirs(nd);
      for (int d = 0; d < nd; ++d) dirs[d] = root + "/" + lname + "-d" + std::to_string(d);
      // slice -> dir, slice lists per worker
      std::vector<std::vector<int>> mine(T);
      std::vector<int> dir_of(nslices);
      const int per_dir = (nslices + nd - 1) / nd;
      for (int i = 0; i < nslices; ++i) {
        if (layout == 0) {
          dir_of[i] = i % nd;
          mine[i % T].push_back(i);
        } else if (layout == 1) {
          dir_of[i] = i / per_dir;
          mine[dir_of[i] % T].push_back(i);
        } else {
          dir_of[i] = i % T;
          mine[i % T].push_back(i);
        }
      }
      auto name = [](int i, int k) { return std::to_string(i) + (k ? "_processed.jpg" : "_original.jpg"); };
      for (int r = 0; r < reps; ++r) {
        for (auto& d : dirs) mkdir(d.c_str(), 0755);
        Phase pw, prw, pwipe, ptmp, pren, preap;
        // cold create
        run(T, pw, [&](int t) {
          std::vector<int> dfd(nd);
          for (int d = 0; d < nd; ++d) dfd[d] = open(dirs[d].c_str(), O_PATH | O_DIRECTORY);
          for (int i : mine[t])
            for (int k = 0; k < 2; ++k) {
              int fd = openat(dfd[dir_of[i]], name(i, k).c_str(), O_WRONLY | O_CREAT | O_EXCL | O_CLOEXEC, 0644);
              if (fd < 0) {
                perror("create");
                abort();
              }
              write_all(fd, src.data() + ((size_t)i * 2 + k) * seg, seg);
              close(fd);
            }
          for (int d : dfd) close(d);
        });
        // warm rewrite
        run(T, prw, [&](int t) {
          std::vector<int> dfd(nd);
          for (int d = 0; d < nd; ++d) dfd[d] = open(dirs[d].c_str(), O_PATH | O_DIRECTORY);
          for (int i : mine[t])
            for (int k = 0; k < 2; ++k) {
              int fd = openat(dfd[dir_of[i]], name(i, k).c_str(), O_WRONLY | O_CLOEXEC);
              if (fd < 0) abort();
              write_all(fd, src.data() + ((size_t)i * 2 + k) * seg, seg);
              close(fd);
            }
          for (int d : dfd) close(d);
        });
        // wipe: whole directories per worker
        run(T, pwipe, [&](int t) {
          for (int d = t; d < nd; d += T) {
            int dfd = open(dirs[d].c_str(), O_RDONLY | O_DIRECTORY);
            DIR* dd = fdopendir(dfd);
            std::vector<std::string> names;
            while (dirent* e = readdir(dd))
              if (e->d_name[0] != '.') names.push_back(e->d_name);
            for (auto& n : names) unlinkat(dfd, n.c_str(), 0);
            closedir(dd);
          }
        });
        // cold export through O_TMPFILE + linkat
        run(T, ptmp, [&](int t) {
          std::vector<int> dfd(nd);
          for (int d = 0; d < nd; ++d) dfd[d] = open(dirs[d].c_str(), O_RDONLY | O_DIRECTORY);
          char proc[64];
          for (int i : mine[t])
            for (int k = 0; k < 2; ++k) {
              int fd = openat(dfd[dir_of[i]], ".", O_TMPFILE | O_WRONLY | O_CLOEXEC, 0644);
              if (fd < 0) {
                perror("O_TMPFILE");
                abort();
              }
              write_all(fd, src.data() + ((size_t)i * 2 + k) * seg, seg);
              int rc = -1;
              if (empty_path_ok != 0) {
                rc = linkat(fd, "", dfd[dir_of[i]], name(i, k).c_str(), AT_EMPTY_PATH);
                if (empty_path_ok < 0) empty_path_ok = rc == 0 ? 1 : 0;
              }
              if (rc != 0) {
                snprintf(proc, sizeof proc, "/proc/self/fd/%d", fd);
                rc = linkat(AT_FDCWD, proc, dfd[dir_of[i]], name(i, k).c_str(), AT_SYMLINK_FOLLOW);
              }
              if (rc != 0) {
                perror("linkat");
                abort();
              }
              close(fd);
            }
          for (int d : dfd) close(d);
        });
        // wipe by renaming each directory into the trash and re-creating it (critical path) ...
        std::atomic<int> seq{0};
        run(T, pren, [&](int t) {
          for (int d = t; d < nd; d += T) {
            std::string dst = trash + "/" + std::to_string(r) + "-" + std::to_string(seq++);
            if (rename(dirs[d].c_str(), dst.c_str()) != 0 || mkdir(dirs[d].c_str(), 0755) != 0) {
              perror("rename");
              abort();
            }
          }
        });
        // ... and the reaper's share: delete what went to the trash (workers take trash dirs)
        std::vector<std::string> sub;
        {
          DIR* td = opendir(trash.c_str());
          while (dirent* e = readdir(td))
            if (e->d_name[0] != '.') sub.push_back(e->d_name);
          closedir(td);
        }
        run(T, preap, [&](int t) {
          for (size_t s = t; s < sub.size(); s += T) {
            std::string p = trash + "/" + sub[s];
            int sfd = open(p.c_str(), O_RDONLY | O_DIRECTORY);
            DIR* sd = fdopendir(sfd);
            std::vector<std::string> names;
            while (dirent* e = readdir(sd))
              if (e->d_name[0] != '.') names.push_back(e->d_name);
            for (auto& n : names) unlinkat(sfd, n.c_str(), 0);
            closedir(sd);
            rmdir(p.c_str());
          }
        });
        auto us = [&](const Phase& p) { return p.cpu.load() / 1e3 / nslices; };
        printf(
            "T=%2d %-7s rep %d | create %6.2f us/slice %7.2f ms | tmpfile %6.2f us %7.2f ms | rewrite %6.2f us %7.2f ms"
            " | wipe %6.2f us %6.2f ms | rename %6.2f ms | reap %6.2f us %6.2f ms\n",
            T, lname, r, us(pw), pw.wall * 1e3, us(ptmp), ptmp.wall * 1e3, us(prw), prw.wall * 1e3, us(pwipe),
            pwipe.wall * 1e3, pren.wall * 1e3, us(preap), preap.wall * 1e3);
        fflush(stdout);
      }
      for (auto& d : dirs) {
        // leave nothing behind: the last rep's tmpfile outputs were moved to the trash and reaped
        rmdir(d.c_str());
      }
    }
  printf("linkat(AT_EMPTY_PATH) for O_TMPFILE: %s\n", empty_path_ok == 1 ? "yes" : "no (/proc/self/fd path)");
  rmdir(trash.c_str());
  rmdir(root.c_str());
  return 0;
}
