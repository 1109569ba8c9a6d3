// gltf_loader.h -- the reference's glTF ingestion (gltf_loader.h:256-810), host side.
//
// Same names and results as the reference so main.cc's sponza() (main.cc:439-498) compiles
// unchanged: gltf::GltfLoader(path).getOutputPrimitives() returns OutputPrimitives with the
// raw little-endian bytes of POSITION / NORMAL / TEXCOORD_0 / TANGENT and of the indices.
// Behaviour kept from the reference:
//  - only buffers[0] is read (gltf_loader.h:563-582), from <dir of the .gltf> + "/" + uri,
//    where <dir> is everything up to the last '/' (empty when the path has none);
//  - every mesh is loaded but each overwrites the previous one, so only the LAST mesh's
//    primitives are returned (gltf_loader.h:295-303);
//  - an accessor's data is count * components * component-bytes contiguous bytes from
//    bufferView.byteOffset + accessor.byteOffset (gltf_loader.h:651-675): byteStride (default
//    1) changes only how the copy is chunked, so interleaved attributes are not de-interleaved;
//  - no node transforms, materials or images are applied.
// Where the reference has undefined behaviour (a missing .bin, an accessor past the end of the
// buffer, a stride chunk overrunning the result) this one throws std::runtime_error instead.
#pragma once
#include <cstdint>
#include <cstring>
#include <fstream>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "json_lite.h"

enum class DataType { kFloat, kByte, kUnsignedByte, kShort, kUnsignedShort, kInt, kUnsignedInt };
enum class PrimitiveMode { kPoints, kLines, kLineLoop, kLineStrip, kTriangles, kTriangleStrip, kTriangleFan };

struct OutputPrimitives {  // gltf_loader.h:40-66
  std::vector<uint8_t> positions, normals, uvs, tangents;
  DataType pos_type = DataType::kFloat, normal_type = DataType::kFloat, uv_type = DataType::kFloat,
           tan_type = DataType::kFloat;
  int pos_comp = 0, normal_comp = 0, uv_comp = 0, tan_comp = 0;
  DataType indices_type = DataType::kUnsignedShort;
  std::vector<uint8_t> indices;
  PrimitiveMode mode = PrimitiveMode::kTriangles;
  bool use_indices = false;
};

namespace gltf {

class GltfLoader {
 public:
  GltfLoader() = default;
  explicit GltfLoader(const std::string& path) : path_(path) {
    doc_ = json_lite::value::parse(read_file(path, "glTF file"));
    data_ = read_buffer0();
    load_last_mesh();
  }
  std::vector<OutputPrimitives>& getOutputPrimitives() { return out_; }

 private:
  std::string path_;
  json_lite::value doc_;
  std::string data_;
  std::vector<OutputPrimitives> out_;

  static std::string read_file(const std::string& p, const char* what) {
    std::ifstream f(p, std::ios::binary);
    if (!f) throw std::runtime_error(std::string("cannot open ") + what + " " + p);
    std::ostringstream ss;
    ss << f.rdbuf();
    return ss.str();
  }
  std::string read_buffer0() const {  // gltf_loader.h:563-582
    const json_lite::value& uri = doc_["buffers"][0]["uri"];
    if (!uri.is_string()) throw std::runtime_error("glTF: buffers[0].uri missing");
    const std::string dir = path_.substr(0, path_.find_last_of('/') + 1);
    return read_file(dir + "/" + uri.as_string(), "glTF buffer");
  }
  static int component_count(const std::string& t) {  // gltf_loader.h:598-616
    if (t == "SCALAR") return 1;
    if (t == "VEC2") return 2;
    if (t == "VEC3") return 3;
    if (t == "VEC4" || t == "MAT2") return 4;
    if (t == "MAT3") return 9;
    if (t == "MAT4") return 16;
    throw std::runtime_error("glTF: unknown accessor type " + t);
  }
  static int component_bytes(int ct) {  // gltf_loader.h:619-629
    if (ct == 5120 || ct == 5121) return 1;
    if (ct == 5122 || ct == 5123) return 2;
    if (ct == 5125 || ct == 5126) return 4;
    throw std::runtime_error("glTF: unknown component type " + std::to_string(ct));
  }
  static DataType data_type(int ct) {  // gltf_loader.h:631-648
    switch (ct) {
      case 5120: return DataType::kByte;
      case 5121: return DataType::kUnsignedByte;
      case 5122: return DataType::kShort;
      case 5123: return DataType::kUnsignedShort;
      case 5125: return DataType::kUnsignedInt;
      case 5126: return DataType::kFloat;
      default: throw std::runtime_error("glTF: unknown component type " + std::to_string(ct));
    }
  }
  // gltf_loader.h:651-675: accessor bytes, contiguous from the view offset plus the accessor offset
  std::vector<uint8_t> accessor_bytes(int index, DataType* type, int* comps) const {
    const json_lite::value& a = doc_["accessors"][(size_t)index];
    if (!a.is_object()) throw std::runtime_error("glTF: accessor " + std::to_string(index) + " missing");
    const int ct = a.value_or("componentType", 0);
    const int n = component_count(a.value_or("type", std::string()));
    const long long len = (long long)a.value_or("count", 0) * n * component_bytes(ct);
    const json_lite::value& view = doc_["bufferViews"][(size_t)a.value_or("bufferView", 0)];
    const long long begin = (long long)view.value_or("byteOffset", 0) + a.value_or("byteOffset", 0);
    if (len < 0 || begin < 0 || begin + len > (long long)data_.size())
      throw std::runtime_error("glTF: accessor " + std::to_string(index) + " reads past the end of buffers[0]");
    std::vector<uint8_t> out((size_t)len);
    if (len) std::memcpy(out.data(), data_.data() + begin, (size_t)len);
    *type = data_type(ct);
    *comps = n;
    return out;
  }
  void load_last_mesh() {  // gltf_loader.h:295-316, 345-389, 540-560
    const json_lite::value& meshes = doc_["meshes"];
    for (size_t m = 0; m < meshes.size(); m++) {
      std::vector<OutputPrimitives> res;
      const json_lite::value& prims = meshes[m]["primitives"];
      for (size_t k = 0; k < prims.size(); k++) {
        const json_lite::value& pr = prims[k];
        const json_lite::value& at = pr["attributes"];
        OutputPrimitives o;
        if (at["POSITION"].is_number())
          o.positions = accessor_bytes((int)at["POSITION"].as_number(), &o.pos_type, &o.pos_comp);
        if (at["NORMAL"].is_number())
          o.normals = accessor_bytes((int)at["NORMAL"].as_number(), &o.normal_type, &o.normal_comp);
        if (at["TEXCOORD_0"].is_number())
          o.uvs = accessor_bytes((int)at["TEXCOORD_0"].as_number(), &o.uv_type, &o.uv_comp);
        if (at["TANGENT"].is_number())
          o.tangents = accessor_bytes((int)at["TANGENT"].as_number(), &o.tan_type, &o.tan_comp);
        const int idx = pr.value_or("indices", -1);
        if (idx != -1) {
          int comps = 0;
          o.indices = accessor_bytes(idx, &o.indices_type, &comps);
          o.use_indices = true;
        }
        const int mode = pr.value_or("mode", 4);
        if (mode < 0 || mode > 6) throw std::runtime_error("glTF: unknown primitive mode " + std::to_string(mode));
        o.mode = (PrimitiveMode)mode;
        res.push_back(std::move(o));
      }
      out_ = std::move(res);  // each mesh replaces the previous one (gltf_loader.h:300-302)
    }
  }
};

}  // namespace gltf
