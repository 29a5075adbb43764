// framework.proto wire reader (ProgramDesc / BlockDesc / VarDesc / OpDesc / Attr) and the
// save_combine tensor stream (.pdiparams) — field numbers as `static/proto.py` / the reference's
// `framework.proto`; no protobuf library.
#include <algorithm>

#include "engine.h"

namespace pdn {

namespace {

struct Reader {
  const uint8_t* p;
  const uint8_t* end;
  Reader(const void* data, size_t n) : p((const uint8_t*)data), end((const uint8_t*)data + n) {}
  bool done() const { return p >= end; }
  uint64_t varint() {
    uint64_t v = 0;
    int shift = 0;
    while (true) {
      if (p >= end) throw std::runtime_error("truncated varint");
      const uint8_t b = *p++;
      v |= (uint64_t)(b & 0x7F) << shift;
      if (!(b & 0x80)) return v;
      shift += 7;
    }
  }
  Reader sub() {
    const uint64_t n = varint();
    if ((size_t)(end - p) < n) throw std::runtime_error("truncated field");
    Reader r(p, n);
    p += n;
    return r;
  }
  std::string str() {
    Reader r = sub();
    return std::string((const char*)r.p, (const char*)r.end);
  }
  void need(size_t n) const {
    if ((size_t)(end - p) < n) throw std::runtime_error("truncated fixed-width field");
  }
  float f32() {
    need(4);
    float f;
    std::memcpy(&f, p, 4);
    p += 4;
    return f;
  }
  double f64() {
    need(8);
    double d;
    std::memcpy(&d, p, 8);
    p += 8;
    return d;
  }
  void skip(int wt) {
    if (wt == 0) varint();
    else if (wt == 1) { need(8); p += 8; }
    else if (wt == 5) { need(4); p += 4; }
    else if (wt == 2) sub();
    else throw std::runtime_error("unsupported wire type");
  }
};

// repeated scalar field: packed (wire type 2) or one element per key
template <typename F>
void repeated(Reader& r, int wt, F&& one) {
  if (wt == 2) {
    Reader s = r.sub();
    while (!s.done()) one(s);
  } else {
    one(r);
  }
}

void parse_tensor_desc(Reader r, VarDesc& v) {
  while (!r.done()) {
    const uint64_t key = r.varint();
    const int f = (int)(key >> 3), wt = (int)(key & 7);
    if (f == 1) v.dtype = (int)r.varint();
    else if (f == 2) repeated(r, wt, [&](Reader& s) { v.dims.push_back((int64_t)s.varint()); });
    else r.skip(wt);
  }
}

void parse_var_type(Reader r, VarDesc& v) {
  while (!r.done()) {
    const uint64_t key = r.varint();
    const int f = (int)(key >> 3), wt = (int)(key & 7);
    if (f == 1) {
      v.type = (int)r.varint();
    } else if (f == 3) {  // lod_tensor: LoDTensorDesc { tensor = 1, lod_level = 2 }
      Reader l = r.sub();
      while (!l.done()) {
        const uint64_t k2 = l.varint();
        if ((k2 >> 3) == 1) parse_tensor_desc(l.sub(), v);
        else l.skip((int)(k2 & 7));
      }
    } else {
      r.skip(wt);
    }
  }
}

VarDesc parse_var(Reader r) {
  VarDesc v;
  while (!r.done()) {
    const uint64_t key = r.varint();
    const int f = (int)(key >> 3), wt = (int)(key & 7);
    if (f == 1) v.name = r.str();
    else if (f == 2) parse_var_type(r.sub(), v);
    else if (f == 3) v.persistable = r.varint() != 0;
    else r.skip(wt);
  }
  return v;
}

void parse_opvar(Reader r, std::map<std::string, std::vector<std::string>>& m) {
  std::string param;
  std::vector<std::string> args;
  while (!r.done()) {
    const uint64_t key = r.varint();
    const int f = (int)(key >> 3), wt = (int)(key & 7);
    if (f == 1) param = r.str();
    else if (f == 2) args.push_back(r.str());
    else r.skip(wt);
  }
  m[param] = std::move(args);
}

std::pair<std::string, Attr> parse_attr(Reader r) {
  std::string name;
  Attr a;
  while (!r.done()) {
    const uint64_t key = r.varint();
    const int f = (int)(key >> 3), wt = (int)(key & 7);
    switch (f) {
      case 1: name = r.str(); break;
      case 2: a.type = (int)r.varint(); break;
      case 3: a.i = (int64_t)(int32_t)r.varint(); break;
      case 4: a.f = r.f32(); break;
      case 5: a.s = r.str(); break;
      case 6: repeated(r, wt, [&](Reader& s) { a.ints.push_back((int64_t)(int32_t)s.varint()); }); break;
      case 7: repeated(r, wt, [&](Reader& s) { a.floats.push_back(s.f32()); }); break;
      case 8: a.strings.push_back(r.str()); break;
      case 10: a.b = r.varint() != 0; break;
      case 11: repeated(r, wt, [&](Reader& s) { a.bools.push_back(s.varint() != 0); }); break;
      case 12: a.i = (int64_t)r.varint(); break;
      case 13: a.i = (int64_t)r.varint(); break;
      case 15: repeated(r, wt, [&](Reader& s) { a.ints.push_back((int64_t)s.varint()); }); break;
      case 16: repeated(r, wt, [&](Reader& s) { a.floats.push_back((float)s.f64()); }); break;
      case 19: a.d = r.f64(); a.f = (float)a.d; break;
      default: r.skip(wt);
    }
  }
  return {name, a};
}

OpDesc parse_op(Reader r) {
  OpDesc op;
  while (!r.done()) {
    const uint64_t key = r.varint();
    const int f = (int)(key >> 3), wt = (int)(key & 7);
    if (f == 3) op.type = r.str();
    else if (f == 1) parse_opvar(r.sub(), op.inputs);
    else if (f == 2) parse_opvar(r.sub(), op.outputs);
    else if (f == 4) op.attrs.insert(parse_attr(r.sub()));
    else r.skip(wt);
  }
  return op;
}

BlockDesc parse_block(Reader r) {
  BlockDesc b;
  while (!r.done()) {
    const uint64_t key = r.varint();
    const int f = (int)(key >> 3), wt = (int)(key & 7);
    if (f == 1) b.idx = (int)r.varint();
    else if (f == 2) b.parent = (int)(int32_t)r.varint();
    else if (f == 3) b.vars.push_back(parse_var(r.sub()));
    else if (f == 4) b.ops.push_back(parse_op(r.sub()));
    else r.skip(wt);
  }
  return b;
}

}  // namespace

ProgramDesc parse_program(const std::string& bytes) {
  ProgramDesc p;
  Reader r(bytes.data(), bytes.size());
  while (!r.done()) {
    const uint64_t key = r.varint();
    const int f = (int)(key >> 3), wt = (int)(key & 7);
    if (f == 1) p.blocks.push_back(parse_block(r.sub()));
    else r.skip(wt);
  }
  std::sort(p.blocks.begin(), p.blocks.end(), [](const BlockDesc& a, const BlockDesc& b) { return a.idx < b.idx; });
  return p;
}

std::unordered_map<std::string, DTensor> load_params(const ProgramDesc& prog, const std::string& bytes) {
  std::vector<std::string> names;
  std::unordered_map<std::string, const VarDesc*> vars;
  for (const auto& v : prog.blocks.at(0).vars) {
    if (v.persistable && v.type == VT_LOD_TENSOR) {
      names.push_back(v.name);
      vars[v.name] = &v;
    }
  }
  std::sort(names.begin(), names.end());
  std::unordered_map<std::string, DTensor> out;
  size_t pos = 0;
  // overflow-safe: n bytes must remain after pos
  auto need = [&](uint64_t n) {
    if (pos > bytes.size() || n > (uint64_t)(bytes.size() - pos))
      throw std::runtime_error("params file truncated or corrupt");
  };
  for (const auto& n : names) {
    if (pos >= bytes.size())  // reference LoadCombine: every persistable must be in the file
      throw std::runtime_error("params file ends before persistable '" + n + "'");
    need(12);
    uint64_t lod_levels;
    std::memcpy(&lod_levels, bytes.data() + pos + 4, 8);
    pos += 12;
    if (lod_levels > 64) throw std::runtime_error("params file: implausible LoD level count");
    for (uint64_t l = 0; l < lod_levels; ++l) {
      need(8);
      uint64_t sz;
      std::memcpy(&sz, bytes.data() + pos, 8);
      pos += 8;
      need(sz);
      pos += sz;
    }
    need(8);
    int32_t dsz;
    std::memcpy(&dsz, bytes.data() + pos + 4, 4);
    pos += 8;
    if (dsz < 0) throw std::runtime_error("params file: negative tensor-desc size");
    need((uint64_t)dsz);
    VarDesc td;
    parse_tensor_desc(Reader(bytes.data() + pos, (size_t)dsz), td);
    pos += (size_t)dsz;
    DTensor t;
    t.dtype = td.dtype;
    t.dims = td.dims;
    for (int64_t d : t.dims)
      if (d < 0 || d > (int64_t(1) << 40)) throw std::runtime_error("params file: bad dims for '" + n + "'");
    const size_t nb = t.nbytes();
    need(nb);
    t.buf = alloc_buffer(nb, false);
    std::memcpy(t.buf->p, bytes.data() + pos, nb);
    pos += nb;
    out[n] = std::move(t);
  }
  if (pos != bytes.size())
    throw std::runtime_error("params file holds " + std::to_string(bytes.size() - pos) +
                             " bytes beyond the program's persistables");
  return out;
}

// ------------------------------------------------------------------------ OpDesc accessors
const std::string& OpDesc::in(const std::string& slot, size_t i) const {
  auto it = inputs.find(slot);
  if (it == inputs.end() || it->second.size() <= i)
    throw std::runtime_error(type + ": missing input " + slot);
  return it->second[i];
}
bool OpDesc::has_in(const std::string& slot) const {
  auto it = inputs.find(slot);
  return it != inputs.end() && !it->second.empty();
}
const std::string& OpDesc::out(const std::string& slot, size_t i) const {
  auto it = outputs.find(slot);
  if (it == outputs.end() || it->second.size() <= i)
    throw std::runtime_error(type + ": missing output " + slot);
  return it->second[i];
}
bool OpDesc::has_out(const std::string& slot) const {
  auto it = outputs.find(slot);
  return it != outputs.end() && !it->second.empty();
}
int64_t OpDesc::ai(const std::string& n, int64_t dflt) const {
  auto it = attrs.find(n);
  if (it == attrs.end()) return dflt;
  if (it->second.type == 6) return it->second.b;
  return it->second.i;
}
float OpDesc::af(const std::string& n, float dflt) const {
  auto it = attrs.find(n);
  if (it == attrs.end()) return dflt;
  if (it->second.type == 0 || it->second.type == 9) return (float)it->second.i;
  return it->second.f;
}
bool OpDesc::ab(const std::string& n, bool dflt) const {
  auto it = attrs.find(n);
  if (it == attrs.end()) return dflt;
  if (it->second.type == 0) return it->second.i != 0;
  return it->second.b;
}
std::string OpDesc::as(const std::string& n, const std::string& dflt) const {
  auto it = attrs.find(n);
  return it == attrs.end() ? dflt : it->second.s;
}
std::vector<int64_t> OpDesc::aints(const std::string& n) const {
  auto it = attrs.find(n);
  return it == attrs.end() ? std::vector<int64_t>{} : it->second.ints;
}

}  // namespace pdn
