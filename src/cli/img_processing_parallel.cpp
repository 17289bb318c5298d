// img_processing_parallel — reference: src/parallel/main_parallel.cpp (main at :389).
// The OpenMP batch-over-images loop (16 threads, batch 25) becomes data-parallel sharding of the
// global patient/slice list over `--gpus N` MI355X ranks (one process per GPU, RCCL over xGMI),
// each rank overlapping DICOM loading, GPU batches and JPEG writing.
// Output: ../out-parallel/PGBM-XXXX/<stem>_{original,processed}.jpg.
#include "nm03/app.h"

int main(int argc, char** argv) {
  nm03::app::AppConfig cfg = nm03::app::parse_args(argc, argv, "img_processing_parallel");
  return nm03::app::cli_exit(nm03::app::run_parallel(cfg));
}
