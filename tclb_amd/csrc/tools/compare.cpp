// tclb-compare: field-by-field comparison of two VTK image datasets (.pvti with its
// .vti pieces, or a single .vti), as written by tclb_amd.io.vtk.
//
//   tclb-compare a.pvti b.pvti [epsilon] [delta_x delta_y delta_z]
//
// Every CellData array present in either file is compared; the maximal absolute
// difference (b sampled at +delta) must not exceed epsilon x machine epsilon of the
// stored type (2.22e-16 Float64, 1.19e-7 Float32, 0 for integer types).  Exit status 0
// when all fields agree.  Behaviour of the reference's tool (src/compare.cpp:242-298);
// written from scratch without an XML library (the files are our own, simple format).
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <set>
#include <sstream>
#include <string>
#include <vector>

namespace {

std::string read_file(const std::string& p) {
  std::ifstream f(p, std::ios::binary);
  if (!f) {
    fprintf(stderr, "cannot open %s\n", p.c_str());
    exit(2);
  }
  std::stringstream ss;
  ss << f.rdbuf();
  return ss.str();
}

std::string attr(const std::string& tag, const std::string& name) {
  const std::string key = " " + name + "=\"";
  size_t i = tag.find(key);
  if (i == std::string::npos) return "";
  i += key.size();
  size_t j = tag.find('"', i);
  return tag.substr(i, j - i);
}

std::vector<uint8_t> b64decode(const char* s, size_t n) {
  static int8_t T[256];
  static bool init = false;
  if (!init) {
    memset(T, -1, sizeof(T));
    const char* a = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
    for (int i = 0; i < 64; i++) T[(uint8_t)a[i]] = (int8_t)i;
    init = true;
  }
  std::vector<uint8_t> out;
  out.reserve(n * 3 / 4);
  uint32_t acc = 0;
  int bits = 0;
  for (size_t i = 0; i < n; i++) {
    const int8_t v = T[(uint8_t)s[i]];
    if (v < 0) continue;   // padding, whitespace
    acc = (acc << 6) | (uint32_t)v;
    bits += 6;
    if (bits >= 8) {
      bits -= 8;
      out.push_back((uint8_t)((acc >> bits) & 0xff));
    }
  }
  return out;
}

struct Field {
  std::string type;
  int ncomp = 1;
  std::vector<double> v;   // (z, y, x, comp), global extent
};

struct Dataset {
  int ext[6] = {0, 0, 0, 0, 0, 0};
  std::map<std::string, Field> fields;
  int nx() const { return ext[1] - ext[0]; }
  int ny() const { return ext[3] - ext[2]; }
  int nz() const { return ext[5] - ext[4]; }
};

double elem(const uint8_t* p, const std::string& t, size_t i) {
  if (t == "Float64") { double v; memcpy(&v, p + 8 * i, 8); return v; }
  if (t == "Float32") { float v; memcpy(&v, p + 4 * i, 4); return v; }
  if (t == "UInt32") { uint32_t v; memcpy(&v, p + 4 * i, 4); return v; }
  if (t == "Int32") { int32_t v; memcpy(&v, p + 4 * i, 4); return v; }
  if (t == "UInt16") { uint16_t v; memcpy(&v, p + 2 * i, 2); return v; }
  if (t == "UInt8") return p[i];
  fprintf(stderr, "unknown field type %s\n", t.c_str());
  exit(2);
}

void read_piece(Dataset& D, const std::string& file) {
  const std::string s = read_file(file);
  size_t pp = s.find("<Piece");
  if (pp == std::string::npos) { fprintf(stderr, "%s: no Piece\n", file.c_str()); exit(2); }
  const std::string ptag = s.substr(pp, s.find('>', pp) - pp);
  int e[6];
  sscanf(attr(ptag, "Extent").c_str(), "%d %d %d %d %d %d", &e[0], &e[1], &e[2], &e[3], &e[4], &e[5]);
  const int pnx = e[1] - e[0], pny = e[3] - e[2], pnz = e[5] - e[4];
  size_t pos = pp;
  while ((pos = s.find("<DataArray", pos)) != std::string::npos) {
    const size_t te = s.find('>', pos);
    const std::string tag = s.substr(pos, te - pos);
    const size_t de = s.find("</DataArray>", te);
    const std::string name = attr(tag, "Name"), type = attr(tag, "type");
    const std::string nc = attr(tag, "NumberOfComponents");
    const int ncomp = nc.empty() ? 1 : atoi(nc.c_str());
    // header (4-byte length) and payload are encoded separately: 8 base64 chars + rest
    size_t b = te + 1;
    while (b < de && isspace((unsigned char)s[b])) b++;
    std::vector<uint8_t> hdr = b64decode(s.data() + b, 8);
    uint32_t nbytes = 0;
    memcpy(&nbytes, hdr.data(), 4);
    std::vector<uint8_t> data = b64decode(s.data() + b + 8, de - b - 8);
    if (data.size() < nbytes) { fprintf(stderr, "%s: truncated %s\n", file.c_str(), name.c_str()); exit(2); }
    Field& F = D.fields[name];
    if (F.v.empty()) {
      F.type = type;
      F.ncomp = ncomp;
      F.v.assign((size_t)D.nx() * D.ny() * D.nz() * ncomp, 0.0);
    }
    for (int z = 0; z < pnz; z++)
      for (int y = 0; y < pny; y++)
        for (int x = 0; x < pnx; x++)
          for (int c = 0; c < ncomp; c++) {
            const size_t li = (((size_t)z * pny + y) * pnx + x) * ncomp + c;
            const size_t gx = x + e[0] - D.ext[0], gy = y + e[2] - D.ext[2], gz = z + e[4] - D.ext[4];
            F.v[(((gz * D.ny()) + gy) * D.nx() + gx) * ncomp + c] = elem(data.data(), type, li);
          }
    pos = de;
  }
}

Dataset load(const std::string& path) {
  Dataset D;
  const std::string s = read_file(path);
  const bool parallel = s.find("PImageData") != std::string::npos;
  const std::string key = parallel ? "<PImageData" : "<ImageData";
  size_t i = s.find(key);
  if (i == std::string::npos) { fprintf(stderr, "%s: not VTK ImageData\n", path.c_str()); exit(2); }
  const std::string tag = s.substr(i, s.find('>', i) - i);
  sscanf(attr(tag, "WholeExtent").c_str(), "%d %d %d %d %d %d", &D.ext[0], &D.ext[1], &D.ext[2], &D.ext[3],
         &D.ext[4], &D.ext[5]);
  printf("%s: %dx%dx%d\n", path.c_str(), D.nx(), D.ny(), D.nz());
  if (!parallel) {
    read_piece(D, path);
    return D;
  }
  const size_t slash = path.find_last_of('/');
  const std::string dir = slash == std::string::npos ? "" : path.substr(0, slash + 1);
  size_t p = i;
  while ((p = s.find("<Piece", p)) != std::string::npos) {
    const std::string ptag = s.substr(p, s.find('>', p) - p);
    std::string src = attr(ptag, "Source");
    if (!src.empty() && src[0] != '/') src = dir + src;
    read_piece(D, src);
    p += 6;
  }
  return D;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 3 || argc > 7 || argc == 5 || argc == 6) {
    printf("usage: tclb-compare file1.pvti file2.pvti [epsilon] [delta_x delta_y delta_z]\n");
    return 2;
  }
  const double eps = argc >= 4 ? atof(argv[3]) : 1e-6;
  const int dx = argc == 7 ? atoi(argv[4]) : 0, dy = argc == 7 ? atoi(argv[5]) : 0, dz = argc == 7 ? atoi(argv[6]) : 0;
  Dataset A = load(argv[1]), B = load(argv[2]);
  printf("Epsilon: %g, Delta: %d, %d, %d\n", eps, dx, dy, dz);
  std::set<std::string> names;
  for (auto& kv : A.fields) names.insert(kv.first);
  for (auto& kv : B.fields) names.insert(kv.first);
  bool ok = true;
  for (const std::string& n : names) {
    if (!A.fields.count(n)) { printf("%s not in first file\n", n.c_str()); ok = false; continue; }
    if (!B.fields.count(n)) { printf("%s not in second file\n", n.c_str()); ok = false; continue; }
    const Field& a = A.fields[n];
    const Field& b = B.fields[n];
    if (a.ncomp != b.ncomp) { printf("%s: component count differs\n", n.c_str()); ok = false; continue; }
    double diff = 0;
    for (int z = 0; z < A.nz(); z++)
      for (int y = 0; y < A.ny(); y++)
        for (int x = 0; x < A.nx(); x++) {
          const int bx = x + dx, by = y + dy, bz = z + dz;
          if (bx < 0 || by < 0 || bz < 0 || bx >= B.nx() || by >= B.ny() || bz >= B.nz()) continue;
          for (int c = 0; c < a.ncomp; c++) {
            const double va = a.v[(((size_t)z * A.ny() + y) * A.nx() + x) * a.ncomp + c];
            const double vb = b.v[(((size_t)bz * B.ny() + by) * B.nx() + bx) * b.ncomp + c];
            const double d = std::fabs(va - vb);
            if (!(d <= diff)) diff = d;   // NaN propagates as a failure
          }
        }
    const double auto_eps = a.type == "Float64" ? 2.22e-16 : (a.type == "Float32" ? 1.19e-07 : 0.0);
    printf("%s: Max difference: %g", n.c_str(), diff);
    if (auto_eps != 0) printf(" = %.1f * %g", diff / auto_eps, auto_eps);
    if (!(diff <= auto_eps * eps)) {
      printf(" --- WRONG\n");
      ok = false;
    } else {
      printf(" --- OK\n");
    }
  }
  return ok ? 0 : 1;
}
