// img_processing_sequential — reference: src/sequential/main_sequential.cpp (main at :346).
// Every patient PGBM-* of the T1+C cohort, one slice at a time (batch 1, one stream), on one
// MI355X. Output: ../out-sequential/PGBM-XXXX/<stem>_{original,processed}.jpg.
#include "nm03/app.h"

int main(int argc, char** argv) {
  nm03::app::AppConfig cfg = nm03::app::parse_args(argc, argv, "img_processing_sequential");
  return nm03::app::cli_exit(nm03::app::run_sequential(cfg));
}
