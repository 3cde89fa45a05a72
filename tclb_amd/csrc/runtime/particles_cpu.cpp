// Host (OpenMP executor) side of the device-resident particle system
// (tclb_amd/particles/system.py): the solid-container builds, the NaN force guard and the
// SimplePart rigid step — the same arithmetic as csrc/device/particles.hip, so the CPU
// executor's Python step path and its native action loop (dist_cpu.cpp) share one
// implementation.  Reference: simplepart.cpp, src/SolidGrid.h, src/SolidTree.hpp:11-120,
// src/Lattice.cu.Rt:420-435.
#include <math.h>

#include <algorithm>
#include <numeric>
#include <vector>

namespace {

long long spread10(long long v) {
  v = (v | (v << 16)) & 0x030000FFLL;
  v = (v | (v << 8)) & 0x0300F00FLL;
  v = (v | (v << 4)) & 0x030C30C3LL;
  return (v | (v << 2)) & 0x09249249LL;
}

double wrap(double x, double L) { return x - floor(x / L) * L; }

}  // namespace

extern "C" {

// grid layout: int header[8] (gx gy gz cell), starts[ncell + 1], ids[n] by cell (stable)
int tclb_part_build_grid_cpu(const double* P, int n, int* grid, int gx, int gy, int gz, int cell, int ncell) {
  if (n <= 0) return 0;
  std::vector<int> cid(n);
  std::vector<int> cnt(ncell + 1, 0);
  const int g[3] = {gx, gy, gz};
  for (int i = 0; i < n; i++) {
    long long c[3];
    for (int d = 0; d < 3; d++) {
      long long v = (long long)floor(P[(long long)i * 10 + d] / (double)cell);
      c[d] = v < 0 ? 0 : (v > g[d] - 1 ? g[d] - 1 : v);
    }
    cid[i] = (int)((c[2] * gy + c[1]) * gx + c[0]);
    cnt[cid[i] + 1]++;
  }
  int acc = 0;
  for (int c = 0; c <= ncell; c++) grid[8 + c] = (acc += cnt[c]);
  std::vector<int> ord(n);
  std::iota(ord.begin(), ord.end(), 0);
  std::stable_sort(ord.begin(), ord.end(), [&](int a, int b) { return cid[a] < cid[b]; });
  for (int i = 0; i < n; i++) grid[9 + ncell + i] = ord[i];
  return 0;
}

// tree layout: int header[8], leaf ids[nl], float boxes[2 nl - 1][6]
int tclb_part_build_tree_cpu(const double* P, int n, int* grid, int nl, double mscale) {
  if (n <= 0) return 0;
  std::vector<long long> code(n);
  for (int i = 0; i < n; i++) {
    long long q[3];
    for (int d = 0; d < 3; d++) {
      double v = P[(long long)i * 10 + d] * mscale;
      v = v < 0.0 ? 0.0 : (v > 1023.0 ? 1023.0 : v);
      q[d] = (long long)v;
    }
    code[i] = spread10(q[0]) | (spread10(q[1]) << 1) | (spread10(q[2]) << 2);
  }
  std::vector<int> ord(n);
  std::iota(ord.begin(), ord.end(), 0);
  std::stable_sort(ord.begin(), ord.end(), [&](int a, int b) { return code[a] < code[b]; });
  float* B = (float*)(grid + 8 + nl);
  for (int j = 0; j < nl; j++) {
    float* b = B + (long long)(nl - 1 + j) * 6;
    if (j < n) {
      grid[8 + j] = ord[j];
      const double* p = P + (long long)ord[j] * 10;
      const double cut = p[9] + 2.05;
      for (int d = 0; d < 3; d++) {
        b[d] = (float)(p[d] - cut);
        b[3 + d] = (float)(p[d] + cut);
      }
    } else {
      grid[8 + j] = -1;
      for (int d = 0; d < 3; d++) {
        b[d] = INFINITY;
        b[3 + d] = -INFINITY;
      }
    }
  }
  int L = 0;
  while ((1 << (L + 1)) <= nl) L++;
  for (int lvl = L - 1; lvl >= 0; lvl--) {
    const int st = (1 << lvl) - 1, cnt = 1 << lvl;
    for (int j = 0; j < cnt; j++) {
      const int i = st + j;
      const float* c0 = B + (long long)(2 * i + 1) * 6;
      const float* c1 = B + (long long)(2 * i + 2) * 6;
      float* b = B + (long long)i * 6;
      for (int d = 0; d < 3; d++) {
        b[d] = std::min(c0[d], c1[d]);
        b[3 + d] = std::max(c0[3 + d], c1[3 + d]);
      }
    }
  }
  return 0;
}

void tclb_part_nan_to_zero_cpu(double* a, int n) {
  for (int i = 0; i < n; i++)
    if (isnan(a[i])) a[i] = 0.0;
}

// v += F/m + a; x += v; omega += T / (2/5 m r^2); periodic wrap of x; fixed particles stay
void tclb_part_rigid_step_cpu(double* P, const double* acc, const double* m, const unsigned char* free_, int n,
                              double ax, double ay, double az, int periodic, double Lx, double Ly, double Lz) {
  for (int i = 0; i < n; i++) {
    if (!free_[i]) continue;
    double* p = P + (long long)i * 10;
    const double* f = acc + (long long)i * 6;
    const double mi = m[i];
    const double vx = p[3] + (f[0] / mi + ax), vy = p[4] + (f[1] / mi + ay), vz = p[5] + (f[2] / mi + az);
    double x = p[0] + vx, y = p[1] + vy, z = p[2] + vz;
    if ((periodic & 1) && Lx > 0) x = wrap(x, Lx);
    if ((periodic & 2) && Ly > 0) y = wrap(y, Ly);
    if ((periodic & 4) && Lz > 0) z = wrap(z, Lz);
    const double I = 0.4 * mi * (p[9] * p[9]);
    p[6] += f[3] / I;
    p[7] += f[4] / I;
    p[8] += f[5] / I;
    p[0] = x;
    p[1] = y;
    p[2] = z;
    p[3] = vx;
    p[4] = vy;
    p[5] = vz;
  }
}

}  // extern "C"
