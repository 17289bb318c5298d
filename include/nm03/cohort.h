// nm03/cohort.h — dataset discovery, slice ordering and output-directory management.
// Reference: SequentialImageProcessor / OptimizedParallelProcessor helpers
//   extractFileNumber        main_sequential.cpp:18-30   (main_parallel.cpp:35-47)
//   setupOutputDirectory     main_sequential.cpp:32-47   (main_parallel.cpp:49-64)
//   findAllPatientDirectories main_sequential.cpp:93-119 (main_parallel.cpp:233-259)
//   loadDICOMFilesForPatient main_sequential.cpp:121-168 (main_parallel.cpp:261-308)
#pragma once

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

namespace nm03::cohort {

// Integer between the last '-' and ".dcm" ("1-14.dcm" → 14); 1000 when absent or unparsable.
int extract_file_number(const std::string& filename);

// Data root: $NM03_DATA_ROOT, else "../data/" (the reference runs from build/).
std::string default_data_root();
std::string with_slash(const std::string& p);
// <root>/Brain-Tumor-Progression/T1-Post-Combined-P001-P020/  (main_sequential.cpp:83-84)
std::string cohort_dir(const std::string& data_root);
// <root>/Brain-Tumor-Progression/PGBM-017/.../1-14.dcm          (test_pipeline.cpp:33-36)
std::string test_slice_path(const std::string& data_root);

// Directories under `cohort_root` whose name starts with "PGBM-", sorted lexicographically.
std::vector<std::string> find_patient_dirs(const std::string& cohort_root);

struct Series {
  std::string series_dir;          // printed as "Using series directory: <dir>/"
  std::vector<std::string> files;  // *.dcm, ordered by extract_file_number then name
};
// Series = lexicographically first sub-directory (the reference takes the first one iterated,
// which is unspecified). Throws std::runtime_error when none exists.
Series list_patient_series(const std::string& cohort_root, const std::string& patient_id);

// mkdir -p <dir> and remove everything inside it (the reference's "mkdir -p && cd && rm -rf *"
// via system(), done with std::filesystem — no shell).
void setup_output_dir(const std::string& dir);
// setup_output_dir for several directories on up to `threads` threads (first error rethrown).
void setup_output_dirs(const std::vector<std::string>& dirs, int threads);
void make_dirs(const std::string& dir);

// The same wipe with the deletion taken off the caller's path. An existing directory is renamed to
// a trash name beside it (".nm03-trash-<pid>-<n>", one rename under the parent's lock) and
// re-created empty at once; `threads` background reaper threads delete the trash while the caller
// goes on (drain() waits for them; the destructor drains too). Trash left behind by a killed run in
// a parent directory is queued as well the first time that parent is seen.
//
// Why (tools/create_probe.cpp on the MI355X box, profiles/r4/create_probe/): creating and deleting
// tmpfs files serialise on per-filesystem locks (inode accounting and the superblock's inode list),
// not on the directory — one-directory-per-thread layouts measure the same. Deleting a JPEG pair
// costs 5–12 µs of CPU on one thread and 23–35 µs with 16 threads deleting at once; done by a few
// reaper threads beside the engine, the wipe costs less CPU and no wall time (4 threads keep up
// with a 465-slice pass every ≈2.3 ms: profiles/r4/cold_ab3/).
class OutputReaper {
 public:
  explicit OutputReaper(int threads = 4);
  ~OutputReaper();
  OutputReaper(const OutputReaper&) = delete;
  OutputReaper& operator=(const OutputReaper&) = delete;
  void wipe(const std::string& dir);  // throws like setup_output_dir
  void wipe(const std::vector<std::string>& dirs);
  void drain();                       // returns when every queued trash directory is gone
  int64_t files_reaped() const;

  struct Impl;

 private:
  std::unique_ptr<Impl> impl_;
};

// File stem ("…/1-14.dcm" → "1-14") and file name.
std::string stem(const std::string& path);
std::string filename(const std::string& path);

}  // namespace nm03::cohort
