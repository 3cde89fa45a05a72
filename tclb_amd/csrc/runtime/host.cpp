// Native host runtime helpers (C ABI, built with g++ -fopenmp into libtclb_host.so).
//
//  * tclb_stl_fill   — STL voxelisation by ray parity along an axis (reference
//                      Geometry::loadSTL, src/Geometry.cpp.Rt:507-688, 'in'/'out' sides)
//  * tclb_stl_cuts   — sub-voxel cut distances Q for the 26 D3Q27 directions and the
//                      surface mask (reference 'surface' side + calcCut, src/Geometry.cpp.Rt:470-505)
//  * tclb_nan_scan   — parallel NaN/Inf scan (Failcheck, src/Handlers/cbFailcheck.cpp:45-93)
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

extern "C" {

// tri: ntri x 9 doubles (p1,p2,p3), already transformed to lattice coords.
// region: global box [x0,x0+nx) x [y0,y0+ny) x [z0,z0+nz) of lev (uint8, x fastest).
// axis: ray axis 0/1/2.  lev[i] starts at insideOut (0/1) and is incremented per hit;
// odd lev = inside.  Returns number of triangle hits.
long long tclb_stl_fill(const double* tri, int ntri, int x0, int y0, int z0, int nx, int ny, int nz, int axis,
                        uint8_t* lev) {
  long long hits = 0;
  const int lo[3] = {x0, y0, z0};
  const int n[3] = {nx, ny, nz};
  const int ax1 = axis, ax2 = (axis + 1) % 3, ax3 = (axis + 2) % 3;
  for (int i = 0; i < ntri; i++) {
    const double* p1 = tri + 9 * i;
    const double* p2 = p1 + 3;
    const double* p3 = p1 + 6;
    int mn[3], mx[3];
    for (int j = 0; j < 3; j++) {
      double a = std::fmin(p1[j], std::fmin(p2[j], p3[j]));
      double b = std::fmax(p1[j], std::fmax(p2[j], p3[j]));
      mn[j] = (int)std::ceil(a) - 1;
      mx[j] = (int)std::floor(b) + 1;
    }
    double v1[2] = {p2[ax2] - p1[ax2], p2[ax3] - p1[ax3]};
    double v2[2] = {p3[ax2] - p1[ax2], p3[ax3] - p1[ax3]};
    double c0 = v1[0] * v2[1] - v1[1] * v2[0];
    if (c0 == 0) continue;
    const double dv[2] = {-0.5694552, 0.8220224};
    double dc1 = (v1[0] * dv[1] - v1[1] * dv[0]) / c0;
    double dc2 = (dv[0] * v2[1] - dv[1] * v2[0]) / c0;
    double dc3 = -dc1 - dc2;
    for (int x2 = mn[ax2]; x2 <= mx[ax2]; x2++)
      for (int x3 = mn[ax3]; x3 <= mx[ax3]; x3++) {
        double v[2] = {x2 - p1[ax2], x3 - p1[ax3]};
        double c1 = (v1[0] * v[1] - v1[1] * v[0]) / c0;
        double c2 = (v[0] * v2[1] - v[1] * v2[0]) / c0;
        double c3 = 1. - c1 - c2;
        int topo = 0;
        if (c1 == 0) { if (dc1 > 0) topo++; } else if (c1 > 0) topo++;
        if (c2 == 0) { if (dc2 > 0) topo++; } else if (c2 > 0) topo++;
        if (c3 == 0) { if (dc3 > 0) topo++; } else if (c3 > 0) topo++;
        if (topo != 3) continue;
        hits++;
        double h = p1[ax1] * c3 + p2[ax1] * c2 + p3[ax1] * c1;
        for (int x1 = lo[ax1]; x1 <= h; x1++) {
          int c[3];
          c[ax1] = x1; c[ax2] = x2; c[ax3] = x3;
          int X = c[0] - x0, Y = c[1] - y0, Z = c[2] - z0;
          if (X < 0 || Y < 0 || Z < 0 || X >= n[0] || Y >= n[1] || Z >= n[2]) continue;
          lev[(size_t)X + (size_t)nx * ((size_t)Y + (size_t)ny * Z)]++;
        }
      }
  }
  return hits;
}

static void gauss4(double* A, double* b, double* x) {
  const int n = 4;
  for (int k = 0; k < n - 1; k++) {
    if (std::fabs(A[k * n + k]) < 1e-10)
      for (int i = k + 1; i < n; i++)
        if (std::fabs(A[i * n + k]) >= 1e-10) {
          for (int j = 0; j < n; j++) std::swap(A[k * n + j], A[i * n + j]);
          std::swap(b[k], b[i]);
          break;
        }
    for (int i = k + 1; i < n; i++) {
      double m = A[i * n + k] / A[k * n + k];
      for (int j = 0; j < n; j++) A[i * n + j] -= m * A[k * n + j];
      b[i] -= m * b[k];
    }
  }
  for (int i = n - 1; i >= 0; i--) {
    double s = 0;
    for (int j = i + 1; j < n; j++) s += A[i * n + j] * x[j];
    x[i] = (b[i] - s) / A[i * n + i];
  }
}

// cut distance (fraction of the link d) from node (x,y,z) along (dx,dy,dz) to the triangle
static double calc_cut(const double* p, double x, double y, double z, int dx, int dy, int dz) {
  // solve  a*(X-p1) + b*(X-p2) + c*(X-p3) = t*d,  a+b+c = 1   (reference calcCut)
  double A[16], b[4] = {0, 0, 0, 1}, r[4];
  const double X[3] = {x, y, z};
  const double d[3] = {(double)dx, (double)dy, (double)dz};
  for (int i = 0; i < 3; i++) {
    A[i * 4 + 0] = X[i] - p[i];
    A[i * 4 + 1] = X[i] - p[3 + i];
    A[i * 4 + 2] = X[i] - p[6 + i];
    A[i * 4 + 3] = d[i];
  }
  A[12] = 1; A[13] = 1; A[14] = 1; A[15] = 0;
  gauss4(A, b, r);
  if (!(r[0] >= 0) || !(r[1] >= 0) || !(r[2] >= 0) || !(r[3] >= 0) || r[3] > 1) return -1;
  return r[3];
}

// Surface voxelisation with cuts.  cuts: uint16 [26][nz][ny][nx] initialised by caller
// to NO_CUT (65535); mask: uint8 [nz][ny][nx] set to 1 where any cut exists.
// dirs: 26 x 3 ints (D3Q27 without rest).  CUT_MAX = 65000.
long long tclb_stl_cuts(const double* tri, int ntri, int x0, int y0, int z0, int nx, int ny, int nz,
                        const int* dirs, uint16_t* cuts, uint8_t* mask) {
  long long nset = 0;
  const size_t plane = (size_t)nx * ny * nz;
  for (int i = 0; i < ntri; i++) {
    const double* p = tri + 9 * i;
    int mn[3], mx[3];
    for (int j = 0; j < 3; j++) {
      double a = std::fmin(p[j], std::fmin(p[3 + j], p[6 + j]));
      double b = std::fmax(p[j], std::fmax(p[3 + j], p[6 + j]));
      mn[j] = (int)std::ceil(a) - 1;
      mx[j] = (int)std::floor(b) + 1;
    }
    for (int x = mn[0]; x <= mx[0]; x++)
      for (int z = mn[2]; z <= mx[2]; z++)
        for (int y = mn[1]; y <= mx[1]; y++) {
          int X = x - x0, Y = y - y0, Z = z - z0;
          if (X < 0 || Y < 0 || Z < 0 || X >= nx || Y >= ny || Z >= nz) continue;
          size_t k = (size_t)X + (size_t)nx * ((size_t)Y + (size_t)ny * Z);
          for (int d = 0; d < 26; d++) {
            double q = calc_cut(p, x, y, z, dirs[3 * d], dirs[3 * d + 1], dirs[3 * d + 2]);
            if (q < 0) continue;
            uint16_t nq = (uint16_t)(q * 65000.0);
            if (nq < cuts[plane * d + k]) cuts[plane * d + k] = nq;
            mask[k] = 1;
            nset++;
          }
        }
  }
  return nset;
}

long long tclb_nan_scan_f64(const double* a, long long n) {
  long long bad = 0;
#pragma omp parallel for reduction(+ : bad)
  for (long long i = 0; i < n; i++) bad += !std::isfinite(a[i]);
  return bad;
}

long long tclb_nan_scan_f32(const float* a, long long n) {
  long long bad = 0;
#pragma omp parallel for reduction(+ : bad)
  for (long long i = 0; i < n; i++) bad += !std::isfinite(a[i]);
  return bad;
}

// Uniform-grid solid container (reference SolidGrid, src/SolidGrid.h:16-179): particles
// binned by centre into cubic cells of edge `cell` (>= max radius + interaction range)
// covering the lattice [0,nx)x[0,ny)x[0,nz); centres outside are clamped into the border
// cells.  Output layout (int32), read by the device ParticleLoop:
//   [0..7]  gx, gy, gz, cell, 0, 0, 0, 0
//   [8 .. 8+ncell]          CSR start of every cell (ncell+1 entries)
//   [9+ncell .. 9+ncell+n)  particle indices sorted by cell
// Returns the number of ints written, or -1 if `cap` is too small.
long long tclb_solid_grid(const double* P, int n, int stride, int nx, int ny, int nz, int cell, int* out,
                          long long cap) {
  if (cell < 1) cell = 1;
  const int gx = (nx + cell - 1) / cell, gy = (ny + cell - 1) / cell, gz = (nz + cell - 1) / cell;
  const long long ncell = (long long)gx * gy * gz;
  const long long need = 8 + ncell + 1 + n;
  if (need > cap) return -1;
  out[0] = gx; out[1] = gy; out[2] = gz; out[3] = cell;
  out[4] = out[5] = out[6] = out[7] = 0;
  int* start = out + 8;
  int* ids = out + 9 + ncell;
  std::vector<int> cid(n);
  for (long long c = 0; c <= ncell; c++) start[c] = 0;
  auto clampi = [](long long v, int hi) { return (int)(v < 0 ? 0 : (v >= hi ? hi - 1 : v)); };
  for (int i = 0; i < n; i++) {
    const double* p = P + (size_t)i * stride;
    const int cx = clampi((long long)std::floor(p[0] / cell), gx);
    const int cy = clampi((long long)std::floor(p[1] / cell), gy);
    const int cz = clampi((long long)std::floor(p[2] / cell), gz);
    cid[i] = (int)(((long long)cz * gy + cy) * gx + cx);
    start[cid[i] + 1]++;
  }
  for (long long c = 0; c < ncell; c++) start[c + 1] += start[c];
  std::vector<int> fill(start, start + ncell);
  for (int i = 0; i < n; i++) ids[fill[cid[i]]++] = i;
  return need;
}

int tclb_host_version() { return 2; }
}
