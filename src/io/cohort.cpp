#include "nm03/cohort.h"

#include <algorithm>
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
  make_dirs(dir);
  std::error_code ec;
  for (const auto& e : fs::directory_iterator(dir, ec)) {
    fs::remove_all(e.path(), ec);
    if (ec) throw std::runtime_error("Failed to setup output directory: " + dir);
  }
  if (ec) throw std::runtime_error("Failed to setup output directory: " + dir);
}

std::string stem(const std::string& path) { return fs::path(path).stem().string(); }
std::string filename(const std::string& path) { return fs::path(path).filename().string(); }

}  // namespace nm03::cohort
