// nm03/metaimage.h — MetaImage (.mhd header + .raw data) writer/reader for stage dumps and golden
// comparisons. The reference includes FAST's MetaImageExporter / ImageFileImporter but never calls
// them (FAST_directives.hpp:29,31); test_pipeline --dump-mhd uses this instead.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace nm03::mhd {

enum class MetType { kUChar, kUShort, kShort, kFloat };

size_t element_size(MetType t);
const char* type_name(MetType t);

// Writes <base>.mhd and <base>.raw (little-endian, uncompressed). d = 1 writes a 2D image.
void write(const std::string& base, const void* data, int w, int h, int d, MetType type, float sx = 1.f,
           float sy = 1.f, float sz = 1.f);

struct Image {
  int w = 0, h = 0, d = 1;
  MetType type = MetType::kUChar;
  float spacing[3] = {1.f, 1.f, 1.f};
  std::vector<uint8_t> bytes;
};
// Reads an .mhd written by write() (or any uncompressed little-endian MetaImage of these types).
Image read(const std::string& mhd_path);

}  // namespace nm03::mhd
