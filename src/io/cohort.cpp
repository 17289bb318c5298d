#include "nm03/cohort.h"

#include <dirent.h>
#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <mutex>
#include <thread>
#include <cstdlib>
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

std::string stem(const std::string& path) { return fs::path(path).stem().string(); }
std::string filename(const std::string& path) { return fs::path(path).filename().string(); }

}  // namespace nm03::cohort
