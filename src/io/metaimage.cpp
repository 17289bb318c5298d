// MetaImage writer/reader (include/nm03/metaimage.h).
#include "nm03/metaimage.h"

#include <fstream>
#include <map>
#include <sstream>
#include <stdexcept>

namespace nm03::mhd {

size_t element_size(MetType t) {
  switch (t) {
    case MetType::kUChar: return 1;
    case MetType::kUShort:
    case MetType::kShort: return 2;
    case MetType::kFloat: return 4;
  }
  return 1;
}

const char* type_name(MetType t) {
  switch (t) {
    case MetType::kUChar: return "MET_UCHAR";
    case MetType::kUShort: return "MET_USHORT";
    case MetType::kShort: return "MET_SHORT";
    case MetType::kFloat: return "MET_FLOAT";
  }
  return "MET_UCHAR";
}

static MetType parse_type(const std::string& s) {
  if (s == "MET_UCHAR") return MetType::kUChar;
  if (s == "MET_USHORT") return MetType::kUShort;
  if (s == "MET_SHORT") return MetType::kShort;
  if (s == "MET_FLOAT") return MetType::kFloat;
  throw std::runtime_error("unsupported MetaImage ElementType " + s);
}

void write(const std::string& base, const void* data, int w, int h, int d, MetType type, float sx, float sy, float sz) {
  const bool is3d = d > 1;
  const std::string raw = base + ".raw";
  const size_t name_at = raw.find_last_of('/');
  const std::string raw_name = name_at == std::string::npos ? raw : raw.substr(name_at + 1);
  std::ofstream hdr(base + ".mhd", std::ios::trunc);
  if (!hdr) throw std::runtime_error("cannot write " + base + ".mhd");
  hdr << "ObjectType = Image\nNDims = " << (is3d ? 3 : 2) << "\nBinaryData = True\n"
      << "BinaryDataByteOrderMSB = False\nCompressedData = False\n"
      << "DimSize = " << w << " " << h << (is3d ? " " + std::to_string(d) : "") << "\n"
      << "ElementSpacing = " << sx << " " << sy;
  if (is3d) hdr << " " << sz;
  hdr << "\nElementType = " << type_name(type) << "\nElementDataFile = " << raw_name << "\n";
  std::ofstream out(raw, std::ios::binary | std::ios::trunc);
  if (!out) throw std::runtime_error("cannot write " + raw);
  out.write((const char*)data, (std::streamsize)((size_t)w * h * (is3d ? d : 1) * element_size(type)));
}

Image read(const std::string& mhd_path) {
  std::ifstream in(mhd_path);
  if (!in) throw std::runtime_error("cannot read " + mhd_path);
  std::map<std::string, std::string> kv;
  std::string line;
  while (std::getline(in, line)) {
    const size_t eq = line.find('=');
    if (eq == std::string::npos) continue;
    auto trim = [](std::string s) {
      const size_t a = s.find_first_not_of(" \t\r"), b = s.find_last_not_of(" \t\r");
      return a == std::string::npos ? std::string() : s.substr(a, b - a + 1);
    };
    kv[trim(line.substr(0, eq))] = trim(line.substr(eq + 1));
  }
  Image img;
  if (kv["CompressedData"] == "True") throw std::runtime_error("compressed MetaImage not supported");
  if (kv["BinaryDataByteOrderMSB"] == "True") throw std::runtime_error("big-endian MetaImage not supported");
  std::istringstream dims(kv["DimSize"]);
  dims >> img.w >> img.h;
  if (!(dims >> img.d)) img.d = 1;
  std::istringstream sp(kv["ElementSpacing"]);
  sp >> img.spacing[0] >> img.spacing[1] >> img.spacing[2];
  img.type = parse_type(kv["ElementType"]);
  std::string raw = kv["ElementDataFile"];
  const size_t slash = mhd_path.find_last_of('/');
  if (!raw.empty() && raw[0] != '/' && slash != std::string::npos) raw = mhd_path.substr(0, slash + 1) + raw;
  std::ifstream r(raw, std::ios::binary);
  if (!r) throw std::runtime_error("cannot read " + raw);
  img.bytes.resize((size_t)img.w * img.h * img.d * element_size(img.type));
  r.read((char*)img.bytes.data(), (std::streamsize)img.bytes.size());
  if ((size_t)r.gcount() != img.bytes.size()) throw std::runtime_error("truncated " + raw);
  return img;
}

}  // namespace nm03::mhd
