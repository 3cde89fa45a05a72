// PNG writer for the headless frames of the colour renderer (the reference opens a GLUT
// window instead: src/gpu_anim.h, Solver::RunMainLoop src/Solver.cpp.Rt:404-427, which
// shows LatticeContainer::Color of a z-slice, src/LatticeContainer.inc.cpp.Rt:350-423).
//
// One RGBA8 image: signature | IHDR | one IDAT (zlib stream of the filtered rows, filter
// type 0) | IEND, each chunk with its CRC-32 (zlib's crc32).
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <zlib.h>

#include <vector>

namespace {

void be32(std::vector<uint8_t>& b, uint32_t v) {
  for (int i = 3; i >= 0; i--) b.push_back((uint8_t)(v >> (8 * i)));
}

void chunk(FILE* fp, const char* type, const uint8_t* data, uint32_t n, bool& ok) {
  std::vector<uint8_t> h;
  be32(h, n);
  h.insert(h.end(), type, type + 4);
  uLong crc = crc32(0L, (const Bytef*)type, 4);
  if (n) crc = crc32(crc, data, n);
  std::vector<uint8_t> t;
  be32(t, (uint32_t)crc);
  ok = ok && fwrite(h.data(), 1, h.size(), fp) == h.size();
  if (n) ok = ok && fwrite(data, 1, n, fp) == n;
  ok = ok && fwrite(t.data(), 1, 4, fp) == 4;
}

}  // namespace

extern "C" {

// rgba: h rows of w pixels (4 bytes each), top row first.  Returns 0, or -1 on error.
int tclb_png_write(const char* path, const uint8_t* rgba, int w, int h) {
  if (w <= 0 || h <= 0) return -1;
  const size_t row = (size_t)w * 4;
  std::vector<uint8_t> raw((row + 1) * (size_t)h);
  for (int y = 0; y < h; y++) {
    raw[(row + 1) * y] = 0;   // filter: none
    memcpy(&raw[(row + 1) * y + 1], rgba + row * y, row);
  }
  uLongf zn = compressBound(raw.size());
  std::vector<uint8_t> z(zn);
  if (compress2(z.data(), &zn, raw.data(), raw.size(), 6) != Z_OK) return -1;
  FILE* fp = fopen(path, "wb");
  if (!fp) return -1;
  static const uint8_t sig[8] = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
  bool ok = fwrite(sig, 1, 8, fp) == 8;
  std::vector<uint8_t> ihdr;
  be32(ihdr, (uint32_t)w);
  be32(ihdr, (uint32_t)h);
  ihdr.push_back(8);   // bit depth
  ihdr.push_back(6);   // colour type RGBA
  ihdr.push_back(0);   // compression
  ihdr.push_back(0);   // filter method
  ihdr.push_back(0);   // no interlace
  chunk(fp, "IHDR", ihdr.data(), (uint32_t)ihdr.size(), ok);
  chunk(fp, "IDAT", z.data(), (uint32_t)zn, ok);
  chunk(fp, "IEND", nullptr, 0, ok);
  ok = (fclose(fp) == 0) && ok;
  return ok ? 0 : -1;
}

}  // extern "C"
