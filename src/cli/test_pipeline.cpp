// test_pipeline — reference: src/test/test_pipeline.cpp (main at :29). One fixed slice through
// every stage; exports original_image, preprocessed_image, segmentation, erosion_result and
// final_dilated_result JPEGs to ../out-test/ (+ a headless 5-view montage). `--cpu` runs the
// golden CPU model (BASELINE config 1).
#include "nm03/app.h"

int main(int argc, char** argv) {
  nm03::app::AppConfig cfg = nm03::app::parse_args(argc, argv, "test_pipeline");
  return nm03::app::cli_exit(nm03::app::run_test_pipeline(cfg));
}
