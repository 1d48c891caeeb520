// loaders.cpp — host asset loaders feeding the scene builder.
//   PlyLoader::load      /root/reference/src/ply_loader.rs:273-430
//   StlLoader::load_binary  stl_loader.rs:10-65
//   ObjLoader::load      obj_loader.rs:332-452
//   Texture::load_png    texture.rs:30-69 (image crate decode + to_rgba8;
//                        here: a small zlib-backed PNG decoder, 8-bit, non-interlaced)
#include <ctype.h>
#include <stdio.h>
#include <string.h>
#include <zlib.h>

#include <algorithm>
#include <array>
#include <fstream>
#include <sstream>

#include "world.h"

namespace massrt {

namespace {

enum class PlyFormat { Ascii, BinaryLE, BinaryBE };
enum class PlyType { Char, UChar, Short, UShort, Int, UInt, Float, Double, Invalid };

PlyType parse_type(const std::string& s) {  // ply_loader.rs:168-186
  if (s == "char" || s == "int8") return PlyType::Char;
  if (s == "uchar" || s == "uint8") return PlyType::UChar;
  if (s == "short" || s == "int16") return PlyType::Short;
  if (s == "ushort" || s == "uint16") return PlyType::UShort;
  if (s == "int" || s == "int32") return PlyType::Int;
  if (s == "uint" || s == "uint32") return PlyType::UInt;
  if (s == "float" || s == "float32") return PlyType::Float;
  if (s == "double" || s == "float64") return PlyType::Double;
  return PlyType::Invalid;
}

size_t type_size(PlyType t) {
  switch (t) {
    case PlyType::Char:
    case PlyType::UChar:
      return 1;
    case PlyType::Short:
    case PlyType::UShort:
      return 2;
    case PlyType::Int:
    case PlyType::UInt:
    case PlyType::Float:
      return 4;
    case PlyType::Double:
      return 8;
    default:
      return 0;
  }
}

struct PlyProp {
  bool is_list;
  std::string name;
  PlyType kind, count_kind;
};
struct PlyElem {
  std::string name;
  size_t count;
  std::vector<PlyProp> props;
};

class Reader {
 public:
  explicit Reader(const std::string& path) : f_(fopen(path.c_str(), "rb")) {
    if (!f_) throw Error(MRT_ERR_IO, "cannot open " + path);
    buf_.resize(1 << 20);
  }
  ~Reader() {
    if (f_) fclose(f_);
  }
  bool getc(unsigned char& c) {
    if (pos_ == len_) {
      len_ = fread(buf_.data(), 1, buf_.size(), f_);
      pos_ = 0;
      if (len_ == 0) return false;
    }
    c = buf_[pos_++];
    return true;
  }
  void read_exact(void* dst, size_t n) {
    unsigned char* d = (unsigned char*)dst;
    for (size_t i = 0; i < n; ++i)
      if (!getc(d[i])) throw Error(MRT_ERR_IO, "unexpected end of file");
  }
  bool read_line(std::string& line) {
    line.clear();
    unsigned char c;
    bool any = false;
    while (getc(c)) {
      any = true;
      line.push_back((char)c);
      if (c == '\n') break;
    }
    return any;
  }
  // ASCII word: skip leading whitespace, stop at the next whitespace
  // (ply_loader.rs:21-32; the terminating whitespace byte is consumed)
  std::string word() {
    std::string w;
    unsigned char c;
    for (;;) {
      if (!getc(c)) throw Error(MRT_ERR_IO, "unexpected end of file");
      if (isspace(c)) {
        if (!w.empty()) break;
      } else {
        w.push_back((char)c);
      }
    }
    return w;
  }

 private:
  FILE* f_;
  std::vector<unsigned char> buf_;
  size_t pos_ = 0, len_ = 0;
};

template <typename T>
T read_bin(Reader& r, bool big_endian) {
  unsigned char b[sizeof(T)];
  r.read_exact(b, sizeof(T));
  if (big_endian)
    for (size_t i = 0; i < sizeof(T) / 2; ++i) std::swap(b[i], b[sizeof(T) - 1 - i]);
  T v;
  memcpy(&v, b, sizeof(T));
  return v;
}

std::string trim(const std::string& s) {
  size_t a = 0, b = s.size();
  while (a < b && isspace((unsigned char)s[a])) ++a;
  while (b > a && isspace((unsigned char)s[b - 1])) --b;
  return s.substr(a, b - a);
}

std::vector<std::string> split_char(const std::string& s, char sep) {
  std::vector<std::string> out;
  size_t start = 0;
  for (;;) {
    size_t p = s.find(sep, start);
    if (p == std::string::npos) {
      out.push_back(s.substr(start));
      return out;
    }
    out.push_back(s.substr(start, p - start));
    start = p + 1;
  }
}

// Rust `str::parse::<usize>()`: optional '+', then ASCII digits only.
bool parse_usize(const std::string& s, uint64_t& out) {
  size_t i = 0;
  if (i < s.size() && s[i] == '+') ++i;
  if (i == s.size()) return false;
  uint64_t v = 0;
  for (; i < s.size(); ++i) {
    if (s[i] < '0' || s[i] > '9') return false;
    uint64_t nv = v * 10 + (uint64_t)(s[i] - '0');
    if (nv / 10 != v) return false;
    v = nv;
  }
  out = v;
  return true;
}

// Rust `str::parse::<f32>()` (correctly rounded) ~ strtof on the whole word.
bool parse_f32(const std::string& s, float& out) {
  if (s.empty()) return false;
  char* end = nullptr;
  std::string t = s;
  out = strtof(t.c_str(), &end);
  return end && *end == '\0';
}

double read_num(Reader& r, PlyFormat fmt, PlyType t) {
  bool be = fmt == PlyFormat::BinaryBE;
  switch (t) {
    case PlyType::Char:
      return (double)read_bin<int8_t>(r, be);
    case PlyType::UChar:
      return (double)read_bin<uint8_t>(r, be);
    case PlyType::Short:
      return (double)read_bin<int16_t>(r, be);
    case PlyType::UShort:
      return (double)read_bin<uint16_t>(r, be);
    case PlyType::Int:
      return (double)read_bin<int32_t>(r, be);
    case PlyType::UInt:
      return (double)read_bin<uint32_t>(r, be);
    case PlyType::Float:
      return (double)read_bin<float>(r, be);
    case PlyType::Double:
      return read_bin<double>(r, be);
    default:
      throw Error(MRT_ERR_IO, "ply: invalid type");
  }
}

// Format::read_f32 (ply_loader.rs:68-111)
float ply_read_f32(Reader& r, PlyFormat fmt, PlyType t) {
  if (fmt == PlyFormat::Ascii) {
    float f;
    if (!parse_f32(r.word(), f)) throw Error(MRT_ERR_IO, "ply: bad float");
    return f;
  }
  if (t == PlyType::Double) return (float)read_num(r, fmt, t);
  if (t == PlyType::Float) return (float)read_num(r, fmt, t);
  return (float)read_num(r, fmt, t);
}

// Format::read_usize (ply_loader.rs:15-66)
uint64_t ply_read_usize(Reader& r, PlyFormat fmt, PlyType t) {
  if (fmt == PlyFormat::Ascii) {
    std::string w = r.word();
    if (t == PlyType::Float || t == PlyType::Double) {
      double d = strtod(w.c_str(), nullptr);
      return d > 0 ? (uint64_t)d : 0;
    }
    uint64_t v;
    if (!parse_usize(w, v)) throw Error(MRT_ERR_IO, "ply: bad integer '" + w + "'");
    return v;
  }
  double d = read_num(r, fmt, t);
  if (t == PlyType::Char || t == PlyType::Short || t == PlyType::Int) return (uint64_t)(int64_t)d;  // `as usize`
  return d > 0 ? (uint64_t)d : 0;
}

void ply_skip(Reader& r, PlyFormat fmt, PlyType t) {
  if (fmt == PlyFormat::Ascii) {
    (void)r.word();
    return;
  }
  unsigned char tmp[8];
  const size_t n = type_size(t);
  if (n > sizeof tmp) throw Error(MRT_ERR_IO, "ply: invalid type");
  r.read_exact(tmp, n);
}

}  // namespace

std::vector<std::array<V3, 3>> load_ply(const std::string& path) {
  return load_ply(path, [](float x, float y, float z) { return V3{x, y, z}; });
}

std::vector<std::array<V3, 3>> load_ply(const std::string& path,
                                        const std::function<V3(float, float, float)>& vertex_fn) {
  Reader r(path);
  std::string line;
  r.read_line(line);
  if (trim(line) != "ply") throw Error(MRT_ERR_IO, "ply magic number not found");
  PlyFormat fmt = PlyFormat::Ascii;
  std::vector<PlyElem> elems;
  for (;;) {
    if (!r.read_line(line)) throw Error(MRT_ERR_IO, "ply: unexpected end of header");
    std::vector<std::string> sp = split_char(trim(line), ' ');
    const std::string& cmd = sp[0];
    if (cmd == "end_header") break;
    if (cmd == "format") {
      std::string f = sp.size() > 1 ? sp[1] : "", v = sp.size() > 2 ? sp[2] : "";
      if (f == "ascii" && v == "1.0")
        fmt = PlyFormat::Ascii;
      else if (f == "binary_little_endian" && v == "1.0")
        fmt = PlyFormat::BinaryLE;
      else if (f == "binary_big_endian" && v == "1.0")
        fmt = PlyFormat::BinaryBE;
      else
        throw Error(MRT_ERR_IO, "ply unsupported format found: " + f + " " + v);
    } else if (cmd == "comment") {
    } else if (cmd == "element") {
      uint64_t count;
      if (sp.size() < 3 || !parse_usize(sp[2], count)) throw Error(MRT_ERR_IO, "ply invalid element: " + line);
      elems.push_back(PlyElem{sp[1], (size_t)count, {}});
    } else if (cmd == "property") {
      if (sp.size() < 2) continue;
      if (sp[1] == "list") {
        PlyType ck = sp.size() > 2 ? parse_type(sp[2]) : PlyType::Invalid;
        PlyType vk = sp.size() > 3 ? parse_type(sp[3]) : PlyType::Invalid;
        if (sp.size() < 5 || ck == PlyType::Invalid || vk == PlyType::Invalid)
          throw Error(MRT_ERR_IO, "ply invalid property: " + line);
        if (!elems.empty()) elems.back().props.push_back(PlyProp{true, sp[4], vk, ck});
      } else {
        PlyType k = parse_type(sp[1]);
        if (sp.size() < 3 || k == PlyType::Invalid) throw Error(MRT_ERR_IO, "ply invalid property: " + line);
        if (!elems.empty()) elems.back().props.push_back(PlyProp{false, sp[2], k, PlyType::Invalid});
      }
    } else if (!cmd.empty()) {
      fprintf(stderr, "unknown ply header found: '%s'\n", cmd.c_str());
    }
  }
  std::vector<V3> verts;
  std::vector<std::array<V3, 3>> faces;
  for (const PlyElem& e : elems) {
    bool is_vertex = e.name == "vertex", is_face = e.name == "face";
    if (is_vertex) verts.reserve(e.count);
    for (size_t i = 0; i < e.count; ++i) {
      bool hx = false, hy = false, hz = false;
      float x = 0, y = 0, z = 0;
      for (const PlyProp& p : e.props) {
        if (!p.is_list) {
          if (is_vertex && p.name == "x") {
            x = ply_read_f32(r, fmt, p.kind), hx = true;
          } else if (is_vertex && p.name == "y") {
            y = ply_read_f32(r, fmt, p.kind), hy = true;
          } else if (is_vertex && p.name == "z") {
            z = ply_read_f32(r, fmt, p.kind), hz = true;
          } else {
            ply_skip(r, fmt, p.kind);
          }
        } else {
          uint64_t count = ply_read_usize(r, fmt, p.count_kind);
          if (is_face && count == 3) {
            uint64_t a = ply_read_usize(r, fmt, p.kind);
            uint64_t b = ply_read_usize(r, fmt, p.kind);
            uint64_t c = ply_read_usize(r, fmt, p.kind);
            if (a >= verts.size() || b >= verts.size() || c >= verts.size())
              throw Error(MRT_ERR_IO, "ply: face index out of range");
            faces.push_back({verts[a], verts[b], verts[c]});
          } else {
            for (uint64_t k = 0; k < count; ++k) ply_skip(r, fmt, p.kind);
          }
        }
      }
      if (is_vertex && hx && hy && hz) verts.push_back(vertex_fn(x, y, z));
    }
  }
  return faces;
}

std::vector<std::array<V3, 3>> load_stl_binary(const std::string& path) {
  Reader r(path);
  unsigned char header[80];
  r.read_exact(header, 80);
  uint32_t n = read_bin<uint32_t>(r, false);
  std::vector<std::array<V3, 3>> faces;
  faces.reserve(n);
  for (uint32_t i = 0; i < n; ++i) {
    float f[12];
    for (int k = 0; k < 12; ++k) f[k] = read_bin<float>(r, false);
    faces.push_back({V3{f[3], f[4], f[5]}, V3{f[6], f[7], f[8]}, V3{f[9], f[10], f[11]}});
    uint16_t attr = read_bin<uint16_t>(r, false);
    std::vector<unsigned char> skip(attr);
    if (attr) r.read_exact(skip.data(), attr);
  }
  return faces;
}

static std::vector<std::string> split_ws(const std::string& s) {
  std::vector<std::string> out;
  std::string cur;
  for (char ch : s) {
    if (isspace((unsigned char)ch)) {
      if (!cur.empty()) out.push_back(cur), cur.clear();
    } else {
      cur.push_back(ch);
    }
  }
  if (!cur.empty()) out.push_back(cur);
  return out;
}

static std::string with_file_name(const std::string& path, const std::string& name) {
  size_t p = path.find_last_of('/');
  return p == std::string::npos ? name : path.substr(0, p + 1) + name;
}

ObjResult load_obj(const std::string& path) {
  std::ifstream in(path);
  if (!in) throw Error(MRT_ERR_IO, "cannot open " + path);
  std::vector<V3> verts, norms;
  std::vector<V2> uvs;
  ObjResult res;
  std::string material;
  std::string line;
  while (std::getline(in, line)) {
    std::vector<std::string> parts = split_ws(line);
    if (parts.empty()) continue;
    const std::string& k = parts[0];
    if (k == "v" || k == "vn") {
      float x, y, z;
      if (parts.size() < 4 || !parse_f32(parts[1], x) || !parse_f32(parts[2], y) || !parse_f32(parts[3], z))
        throw Error(MRT_ERR_IO, "unable to parse vertex: " + line);
      (k == "v" ? verts : norms).push_back(V3{x, y, z});
    } else if (k == "vt") {
      float u, v;
      if (parts.size() < 3 || !parse_f32(parts[1], u) || !parse_f32(parts[2], v))
        throw Error(MRT_ERR_IO, "unable to parse texture coord: " + line);
      uvs.push_back(V2{u, v});
    } else if (k == "f") {
      // obj_loader.rs:398-429: only the first three corners; `v//vn` borrows uvs[0]
      ObjFace face;
      for (int c = 0; c < 3; ++c) {
        if ((size_t)(c + 1) >= parts.size()) throw Error(MRT_ERR_IO, "unable to parse face: " + line);
        const std::string& s = parts[c + 1];
        std::vector<uint64_t> idx;
        for (const std::string& t : split_char(s, '/')) {
          uint64_t v;
          if (parse_usize(t, v)) idx.push_back(v);
        }
        bool dbl = s.find("//") != std::string::npos;
        bool ok;
        if (dbl) {
          ok = idx.size() >= 2 && idx[0] >= 1 && idx[0] <= verts.size() && !uvs.empty() && idx[1] >= 1 &&
               idx[1] <= norms.size();
          if (ok) face.c[c] = ObjCorner{verts[idx[0] - 1], norms[idx[1] - 1], uvs[0]};
        } else {
          ok = idx.size() >= 3 && idx[0] >= 1 && idx[0] <= verts.size() && idx[1] >= 1 && idx[1] <= uvs.size() &&
               idx[2] >= 1 && idx[2] <= norms.size();
          if (ok) face.c[c] = ObjCorner{verts[idx[0] - 1], norms[idx[2] - 1], uvs[idx[1] - 1]};
        }
        if (!ok) throw Error(MRT_ERR_IO, "unable to parse face: " + line);
      }
      face.material = material;
      res.faces.push_back(face);
    } else if (k == "usemtl") {
      if (parts.size() > 1) material = parts[1];
    } else if (k == "mtllib") {
      std::string name;
      for (size_t i = 1; i < parts.size(); ++i) name += (i > 1 ? " " : "") + parts[i];
      res.material_library = with_file_name(path, name);
    }
  }
  return res;
}

// ---- PNG ------------------------------------------------------------------
static uint32_t be32(const unsigned char* p) { return (uint32_t)p[0] << 24 | p[1] << 16 | p[2] << 8 | p[3]; }

bool decode_png(const std::string& path, std::vector<uint8_t>& rgba, uint32_t& w, uint32_t& h, std::string& err) {
  std::ifstream in(path, std::ios::binary);
  if (!in) {
    err = "cannot open " + path;
    return false;
  }
  std::vector<unsigned char> data((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
  static const unsigned char sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
  if (data.size() < 8 || memcmp(data.data(), sig, 8) != 0) {
    err = "not a PNG file";
    return false;
  }
  size_t p = 8;
  uint32_t depth = 0, ctype = 0, interlace = 0;
  std::vector<unsigned char> idat, plte, trns;
  while (p + 8 <= data.size()) {
    uint32_t len = be32(&data[p]);
    std::string type((const char*)&data[p + 4], 4);
    if (p + 12 + (size_t)len > data.size()) break;
    const unsigned char* c = &data[p + 8];
    if (type == "IHDR") {
      w = be32(c), h = be32(c + 4), depth = c[8], ctype = c[9], interlace = c[12];
    } else if (type == "PLTE") {
      plte.assign(c, c + len);
    } else if (type == "tRNS") {
      trns.assign(c, c + len);
    } else if (type == "IDAT") {
      idat.insert(idat.end(), c, c + len);
    } else if (type == "IEND") {
      break;
    }
    p += 12 + len;
  }
  int ch = ctype == 0 ? 1 : ctype == 2 ? 3 : ctype == 3 ? 1 : ctype == 4 ? 2 : ctype == 6 ? 4 : 0;
  bool sub_byte_ok = (ctype == 0 || ctype == 3) && (depth == 1 || depth == 2 || depth == 4);
  if (!ch || interlace != 0 || !(depth == 8 || sub_byte_ok)) {
    err = "unsupported PNG (need 8-bit, or 1/2/4-bit gray/palette; non-interlaced)";
    return false;
  }
  const size_t stride = ((size_t)w * ch * depth + 7) / 8;
  const size_t bpp = std::max<size_t>(1, (size_t)ch * depth / 8);
  std::vector<unsigned char> raw((stride + 1) * h);
  uLongf rawlen = raw.size();
  if (uncompress(raw.data(), &rawlen, idat.data(), idat.size()) != Z_OK || rawlen != raw.size()) {
    err = "PNG inflate failed";
    return false;
  }
  std::vector<unsigned char> img(stride * h), prev(stride, 0);
  for (uint32_t y = 0; y < h; ++y) {
    unsigned char f = raw[y * (stride + 1)];
    unsigned char* src = &raw[y * (stride + 1) + 1];
    unsigned char* dst = &img[y * stride];
    for (size_t x = 0; x < stride; ++x) {
      int a = x >= bpp ? dst[x - bpp] : 0, b = prev[x], cc = x >= bpp ? prev[x - bpp] : 0;
      int pred = 0;
      if (f == 1) pred = a;
      else if (f == 2) pred = b;
      else if (f == 3) pred = (a + b) / 2;
      else if (f == 4) {
        int pp = a + b - cc, pa = abs(pp - a), pb = abs(pp - b), pc = abs(pp - cc);
        pred = (pa <= pb && pa <= pc) ? a : (pb <= pc ? b : cc);
      } else if (f != 0) {
        err = "bad PNG filter";
        return false;
      }
      dst[x] = (unsigned char)(src[x] + pred);
    }
    memcpy(prev.data(), dst, stride);
  }
  auto sample = [&](uint32_t y, size_t i) -> unsigned {  // i-th sample of row y
    if (depth == 8) return img[y * stride + i];
    size_t bit = i * depth;
    unsigned byte = img[y * stride + bit / 8];
    return (byte >> (8 - depth - bit % 8)) & ((1u << depth) - 1);
  };
  const unsigned maxv = (1u << depth) - 1;
  rgba.resize((size_t)w * h * 4);
  for (uint32_t y = 0; y < h; ++y)
    for (uint32_t x = 0; x < w; ++x) {
      unsigned char* o = &rgba[4 * ((size_t)y * w + x)];
      size_t i0 = (size_t)x * ch;
      switch (ctype) {
        case 0: {
          unsigned v = sample(y, i0);
          o[0] = o[1] = o[2] = (unsigned char)(v * 255 / maxv);
          o[3] = (trns.size() >= 2 && v == (unsigned)(trns[0] << 8 | trns[1])) ? 0 : 255;
          break;
        }
        case 2:
          o[0] = (unsigned char)sample(y, i0), o[1] = (unsigned char)sample(y, i0 + 1),
          o[2] = (unsigned char)sample(y, i0 + 2);
          o[3] = (trns.size() >= 6 && o[0] == trns[1] && o[1] == trns[3] && o[2] == trns[5]) ? 0 : 255;
          break;
        case 3: {
          size_t k = sample(y, i0);
          if (3 * k + 2 >= plte.size()) {
            err = "PNG palette index out of range";
            return false;
          }
          o[0] = plte[3 * k], o[1] = plte[3 * k + 1], o[2] = plte[3 * k + 2], o[3] = k < trns.size() ? trns[k] : 255;
          break;
        }
        case 4:
          o[0] = o[1] = o[2] = (unsigned char)sample(y, i0), o[3] = (unsigned char)sample(y, i0 + 1);
          break;
        default:
          for (int k = 0; k < 4; ++k) o[k] = (unsigned char)sample(y, i0 + k);
      }
    }
  return true;
}

SharedTexture Texture::load_png(const std::string& path, WrapMode wrapping) {
  auto t = std::make_shared<Texture>();
  std::string err;
  if (!decode_png(path, t->rgba, t->width, t->height, err)) throw Error(MRT_ERR_IO, err);
  t->wrapping = wrapping;
  return t;
}

SharedTexture Texture::load_bytes(const uint8_t* bytes, uint32_t w, uint32_t h, WrapMode wrapping) {
  auto t = std::make_shared<Texture>();
  t->width = w;
  t->height = h;
  t->wrapping = wrapping;
  t->rgba.assign(bytes, bytes + (size_t)w * h * 4);
  return t;
}

}  // namespace massrt
