#include "nm03/cohort.h"

#include <dirent.h>
#include <fcntl.h>
#include <linux/capability.h>
#include <pthread.h>
#include <signal.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <set>
#include <thread>
#include <cstdlib>
#include <cstring>
#include <filesystem>
#include <stdexcept>
#include <system_error>

namespace fs = std::filesystem;

namespace nm03::cohort {

int extract_file_number(const std::string& name) {
  // Same semantics as the reference: find_last_of('-'), find(".dcm"), std::stoi (which accepts a
  // numeric prefix and throws when there is none) with a 1000 fallback.
  size_t dash = name.find_last_of('-');
  size_t dot = name.find(".dcm");
  if (dash != std::string::npos && dot != std::string::npos) {
    std::string num = name.substr(dash + 1, dot - dash - 1);
    try {
      return std::stoi(num);
    } catch (...) {
      return 1000;
    }
  }
  return 1000;
}

std::string with_slash(const std::string& p) {
  if (p.empty() || p.back() == '/') return p;
  return p + "/";
}

std::string default_data_root() {
  const char* e = std::getenv("NM03_DATA_ROOT");
  if (e && *e) return with_slash(e);
  return "../data/";
}

std::string cohort_dir(const std::string& data_root) {
  return with_slash(data_root) + "Brain-Tumor-Progression/T1-Post-Combined-P001-P020/";
}

std::string test_slice_path(const std::string& data_root) {
  return with_slash(data_root) +
         "Brain-Tumor-Progression/PGBM-017/09-17-1997-RA FH MR RCBV OP-85753/16.000000-T1post-19554/1-14.dcm";
}

std::vector<std::string> find_patient_dirs(const std::string& cohort_root) {
  std::vector<std::string> out;
  for (const auto& e : fs::directory_iterator(cohort_root)) {
    if (!e.is_directory()) continue;
    std::string name = e.path().filename().string();
    if (name.rfind("PGBM-", 0) == 0) out.push_back(name);
  }
  std::sort(out.begin(), out.end());
  return out;
}

Series list_patient_series(const std::string& cohort_root, const std::string& patient_id) {
  const std::string patient_path = with_slash(cohort_root) + patient_id + "/";
  std::vector<std::string> series_dirs;
  for (const auto& e : fs::directory_iterator(patient_path))
    if (e.is_directory()) series_dirs.push_back(e.path().string() + "/");
  if (series_dirs.empty()) throw std::runtime_error("No series directories found for patient: " + patient_id);
  std::sort(series_dirs.begin(), series_dirs.end());
  Series s;
  s.series_dir = series_dirs[0];
  std::vector<std::pair<int, std::string>> files;
  for (const auto& e : fs::directory_iterator(s.series_dir)) {
    if (e.path().extension() == ".dcm")
      files.push_back({extract_file_number(e.path().filename().string()), e.path().string()});
  }
  std::sort(files.begin(), files.end());
  for (auto& f : files) s.files.push_back(std::move(f.second));
  return s;
}

void make_dirs(const std::string& dir) {
  std::error_code ec;
  fs::create_directories(dir, ec);
  if (ec && !fs::is_directory(dir)) throw std::runtime_error("Failed to create directory: " + dir + " (" + ec.message() + ")");
}

void setup_output_dir(const std::string& dir) {
  // The reference's `mkdir -p dir && cd dir && rm -rf *` (main_sequential.cpp:32-47) without a
  // shell: names listed first, then one unlinkat per file (std::filesystem::remove_all costs
  // several stat calls per entry); subdirectories go through remove_all.
  make_dirs(dir);
  const int dfd = ::open(dir.c_str(), O_RDONLY | O_DIRECTORY | O_CLOEXEC);
  if (dfd < 0) throw std::runtime_error("Failed to setup output directory: " + dir);
  DIR* d = ::fdopendir(dfd);
  if (!d) {
    ::close(dfd);
    throw std::runtime_error("Failed to setup output directory: " + dir);
  }
  std::vector<std::string> files, subdirs;
  while (dirent* e = ::readdir(d)) {
    const char* nm = e->d_name;
    if (nm[0] == '.' && (nm[1] == 0 || (nm[1] == '.' && nm[2] == 0))) continue;
    (e->d_type == DT_DIR ? subdirs : files).push_back(nm);
  }
  bool ok = true;
  for (const auto& f : files)
    if (::unlinkat(dfd, f.c_str(), 0) != 0) {
      if (errno == EISDIR)
        subdirs.push_back(f);
      else if (errno != ENOENT)
        ok = false;
    }
  ::closedir(d);  // closes dfd
  std::error_code ec;
  for (const auto& sd : subdirs) {
    fs::remove_all(fs::path(dir) / sd, ec);
    if (ec) ok = false;
  }
  if (!ok) throw std::runtime_error("Failed to setup output directory: " + dir);
}

void setup_output_dirs(const std::vector<std::string>& dirs, int threads) {
  std::atomic<size_t> next{0};
  std::string err;
  std::mutex m;
  auto work = [&] {
    for (size_t i; (i = next.fetch_add(1)) < dirs.size();) {
      try {
        setup_output_dir(dirs[i]);
      } catch (const std::exception& e) {
        std::lock_guard<std::mutex> g(m);
        if (err.empty()) err = e.what();
      }
    }
  };
  const int nt = std::max(1, std::min<int>(threads, (int)dirs.size()));
  std::vector<std::thread> th;
  for (int t = 1; t < nt; ++t) th.emplace_back(work);
  work();
  for (auto& t : th) t.join();
  if (!err.empty()) throw std::runtime_error(err);
}

namespace {

// Deletes everything under `dir` and `dir` itself; returns the number of files unlinked.
int64_t remove_tree(const std::string& dir) {
  const int dfd = ::open(dir.c_str(), O_RDONLY | O_DIRECTORY | O_CLOEXEC);
  if (dfd < 0) return 0;
  DIR* d = ::fdopendir(dfd);
  if (!d) {
    ::close(dfd);
    return 0;
  }
  std::vector<std::string> files, subdirs;
  while (dirent* e = ::readdir(d)) {
    const char* nm = e->d_name;
    if (nm[0] == '.' && (nm[1] == 0 || (nm[1] == '.' && nm[2] == 0))) continue;
    (e->d_type == DT_DIR ? subdirs : files).push_back(nm);
  }
  int64_t n = 0;
  for (const auto& f : files) {
    if (::unlinkat(dfd, f.c_str(), 0) == 0)
      ++n;
    else if (errno == EISDIR)
      subdirs.push_back(f);
  }
  ::closedir(d);
  for (const auto& sd : subdirs) n += remove_tree(dir + "/" + sd);
  ::rmdir(dir.c_str());
  return n;
}

constexpr const char* kTrashPrefix = ".nm03-trash-";

}  // namespace

struct OutputReaper::Impl {
  std::mutex m;
  std::condition_variable cv, idle_cv;
  std::deque<std::string> q;
  size_t busy = 0;
  bool stop = false;
  std::atomic<int64_t> files{0};
  std::atomic<uint64_t> seq{0};
  std::set<std::string> parents_seen;  // guarded by m
  std::vector<std::thread> threads;

  void push(std::string p) {
    {
      std::lock_guard<std::mutex> g(m);
      q.push_back(std::move(p));
    }
    cv.notify_one();
  }
  void run() {
    pthread_setname_np(pthread_self(), "nm03-reaper");
    // Own fd table and cred, like the engine's pool workers (engine.cpp): no shared fd-table lock
    // or cred refcount line with the writers.
#ifndef CLOSE_RANGE_UNSHARE
#define CLOSE_RANGE_UNSHARE (1U << 1)
#endif
    (void)::syscall(SYS_close_range, 3u, ~0u, CLOSE_RANGE_UNSHARE);
    __user_cap_header_struct h{_LINUX_CAPABILITY_VERSION_3, 0};
    __user_cap_data_struct c[2]{};
    if (::syscall(SYS_capget, &h, c) == 0) (void)::syscall(SYS_capset, &h, c);
    for (;;) {
      std::string p;
      {
        std::unique_lock<std::mutex> g(m);
        cv.wait(g, [&] { return stop || !q.empty(); });
        if (q.empty()) return;
        p = std::move(q.front());
        q.pop_front();
        ++busy;
      }
      files += remove_tree(p);
      {
        std::lock_guard<std::mutex> g(m);
        --busy;
        if (q.empty() && busy == 0) idle_cv.notify_all();
      }
    }
  }
  // Stale trash of killed runs in `parent` (first time the parent is seen): only entries whose
  // owner (the pid in ".nm03-trash-<pid>-<seq>") is gone. A live run's trash — another process
  // writing to the same output root, or another reaper of this one — is its own reaper's to delete.
  static bool owner_alive(const char* name) {
    const char* p = name + std::strlen(kTrashPrefix);
    char* end = nullptr;
    const long pid = std::strtol(p, &end, 10);
    if (end == p || *end != '-' || pid <= 0) return false;  // not ours: treat as stale
    if (pid == (long)::getpid()) return true;
    return ::kill((pid_t)pid, 0) == 0 || errno != ESRCH;
  }
  void sweep_parent(const std::string& parent) {
    {
      std::lock_guard<std::mutex> g(m);
      if (!parents_seen.insert(parent).second) return;
    }
    DIR* d = ::opendir(parent.c_str());
    if (!d) return;
    std::vector<std::string> stale;
    while (dirent* e = ::readdir(d))
      if (std::strncmp(e->d_name, kTrashPrefix, std::strlen(kTrashPrefix)) == 0 && !owner_alive(e->d_name))
        stale.push_back(e->d_name);
    ::closedir(d);
    for (auto& n : stale) push(parent + "/" + n);
  }
};

OutputReaper::OutputReaper(int threads) : impl_(std::make_unique<Impl>()) {
  for (int t = 0; t < std::max(1, threads); ++t) impl_->threads.emplace_back([this] { impl_->run(); });
}

OutputReaper::~OutputReaper() {
  drain();
  {
    std::lock_guard<std::mutex> g(impl_->m);
    impl_->stop = true;
  }
  impl_->cv.notify_all();
  for (auto& t : impl_->threads) t.join();
}

void OutputReaper::wipe(const std::string& dir_in) {
  std::string dir = dir_in;
  while (dir.size() > 1 && dir.back() == '/') dir.pop_back();
  const size_t slash = dir.rfind('/');
  const std::string parent = slash == std::string::npos ? "." : slash == 0 ? "/" : dir.substr(0, slash);
  make_dirs(parent);
  impl_->sweep_parent(parent);
  const std::string trash = parent + "/" + kTrashPrefix + std::to_string(::getpid()) + "-" +
                            std::to_string(impl_->seq.fetch_add(1));
  if (::rename(dir.c_str(), trash.c_str()) == 0) {
    impl_->push(trash);
  } else if (errno != ENOENT) {
    setup_output_dir(dir);  // not renamable (a mount point, another file system): wipe in place
    return;
  }
  if (::mkdir(dir.c_str(), 0755) != 0 && errno != EEXIST)
    throw std::runtime_error("Failed to setup output directory: " + dir + " (" + std::strerror(errno) + ")");
}

void OutputReaper::wipe(const std::vector<std::string>& dirs) {
  for (const auto& d : dirs) wipe(d);
}

void OutputReaper::drain() {
  std::unique_lock<std::mutex> g(impl_->m);
  impl_->idle_cv.wait(g, [&] { return impl_->q.empty() && impl_->busy == 0; });
}

int64_t OutputReaper::files_reaped() const { return impl_->files.load(); }

std::string stem(const std::string& path) { return fs::path(path).stem().string(); }
std::string filename(const std::string& path) { return fs::path(path).filename().string(); }

}  // namespace nm03::cohort
