// frei_binning.hip — K6: binning of high-resolution opacity cross-sections onto a grid's
// wavelength bins (frei/opacity.py:66-170 binned_opacity; frei/interp.py:156-307
// groupby_bins_agg + AggregateTrapz; opacity.py:33-42 mapfunc_exact).
//
// Data: one species' cross-section stays resident in HBM as float32
// [n_T][n_p][n_hi] (the opacity_dir_to_netcdf layout, opacity.py:395-483).  The host
// side (C++, this file) builds the row-independent plan once per call — pandas.cut bin
// ranges over the ascending high-res axis, nearest source node per target (T, p) node,
// group coordinates and interpolation brackets — and the kernels do the row-dependent
// streaming work:
//   groupies (default of binned_opacity): one lane per (source row, bin) walks its bin's
//     points in order with the reference's float32 accumulator and fans the result out
//     to every destination (p, T) row that selected this source row (no intermediate);
//   exact (Grid.load_opacities default): a block of 256 grid wavelengths integrates the
//     non-empty bins its interpolation brackets span into LDS, a source-row batch at a time,
//     then each lane interpolates linearly and fans its value out the same way (no
//     intermediate array).
// Both are HBM-bound streams: float32 reads of the selected source rows + float64 writes
// of the destination table, the writes streaming (non-temporal).
#include <algorithm>
#include <cmath>
#include <cstring>
#include <map>
#include <numeric>
#include <string>
#include <vector>

#include "../../include/frei_hip.h"
#include "frei_device.h"

using namespace frei;

struct frei_xsec {
  int device = 0;
  hipStream_t stream = nullptr;
  int nT = 0, np = 0;
  int64_t nhi = 0;
  std::vector<double> T, p, wl;  // K, bar, µm (ascending)
  float* d_x = nullptr;          // [nT][np][nhi]
  double* d_hdx = nullptr;       // 0.5 * (wl[i+1] - wl[i]), exact mode (lazy)
  double* d_scratch = nullptr;   // output of frei_xsec_bin(out = NULL)
  size_t scratch_n = 0;
  bool timing = false;
  double t_ms = 0;
  int t_n = 0;
  // the per-call plan arrays, kept between calls (slot k: device buffer and its capacity in
  // bytes): no hipMalloc / hipFree per binning call
  std::vector<std::pair<void*, size_t>> plan;
  // pinned host staging of the plan uploads (DMA copies; pageable hipMemcpyAsync stalled the
  // next kernel launch by milliseconds)
  char* pinned = nullptr;
  size_t pinned_cap = 0, pinned_used = 0;
};

namespace {

constexpr int kExactRows = 8;     // source rows per block in the exact mode
constexpr int kGroupiesRows = 8;  // source rows per lane in the groupies pass
constexpr int kGroupiesBatch = 4; // of which summed together (loads in flight)

#define HIP_TRY(expr)                                                                   \
  do {                                                                                  \
    hipError_t _e = (expr);                                                             \
    if (_e != hipSuccess) return set_error(std::string(#expr) + ": " + hipGetErrorString(_e)); \
  } while (0)
#define TRY(expr)            \
  do {                       \
    int _r = (expr);         \
    if (_r != 0) return _r;  \
  } while (0)

template <typename T>
int dalloc(T** p, size_t n) {
  if (n == 0) n = 1;
  HIP_TRY(hipMalloc((void**)p, n * sizeof(T)));
  return 0;
}
template <typename T>
void dfree(T*& p) {
  if (p) (void)hipFree((void*)p);
  p = nullptr;
}
// Plan array `slot` of x on the device (grown when too small) holding h.
template <typename T>
int stage(frei_xsec* x, int slot, T** d, const std::vector<T>& h, hipStream_t st) {
  if ((int)x->plan.size() <= slot) x->plan.resize(slot + 1, {nullptr, 0});
  auto& b = x->plan[slot];
  const size_t need = std::max<size_t>(h.size(), 1) * sizeof(T);
  if (b.second < need) {
    if (b.first) (void)hipFree(b.first);
    b = {nullptr, 0};
    HIP_TRY(hipMalloc(&b.first, need));
    b.second = need;
  }
  *d = static_cast<T*>(b.first);
  if (h.empty()) return 0;
  const size_t n = h.size() * sizeof(T);
  const size_t at = (x->pinned_used + 255) & ~size_t(255);
  if (at + n > x->pinned_cap) return set_error("binning: plan staging buffer too small");
  std::memcpy(x->pinned + at, h.data(), n);
  x->pinned_used = at + n;
  HIP_TRY(hipMemcpyAsync(*d, x->pinned + at, n, hipMemcpyHostToDevice, st));
  return 0;
}
// Room for `bytes` of plan uploads in x's pinned staging buffer.  The stream is synchronised
// first: no copy out of the buffer may still be in flight when it is reused or freed (every
// bin_into path already ends synchronised; this keeps the invariant local).
int stage_reserve(frei_xsec* x, size_t bytes) {
  HIP_TRY(hipStreamSynchronize(x->stream));
  x->pinned_used = 0;
  if (bytes <= x->pinned_cap) return 0;
  if (x->pinned) (void)hipHostFree(x->pinned);
  x->pinned = nullptr;
  x->pinned_cap = 0;
  HIP_TRY(hipHostMalloc((void**)&x->pinned, bytes, hipHostMallocDefault));
  x->pinned_cap = bytes;
  return 0;
}
template <typename T>
int upload(T** d, const std::vector<T>& h, hipStream_t st) {
  TRY(dalloc(d, h.size()));
  if (!h.empty()) HIP_TRY(hipMemcpyAsync(*d, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice, st));
  return 0;
}

// ------------------------------------------------------------------- kernels
// groupies: AggregateTrapz._loop (interp.py:176-194) with dx = 1 for one (row, bin):
// acc_f32 = f32(f64(acc_f32) + f64(f32(a_i + a_{i+1})) / 2) over consecutive pairs of the
// bin in point order (numba promotion, float32 result array), then
// (f64(acc) * (b_{k+1} - b_k)) * 1e-3 (opacity.py:136-139), stored to every destination
// row of this source row.  One lane per bin loops over source rows [u0, u1) so the bin's
// range and width are read once per lane, not once per row.
__global__ __launch_bounds__(256) void bin_groupies_kernel(
    const float* __restrict__ x, const int64_t* __restrict__ row_off, int U, int rows_per,
    const int64_t* __restrict__ start, const int64_t* __restrict__ end,
    const double* __restrict__ width, int64_t nb, const int32_t* __restrict__ fan_off,
    const int64_t* __restrict__ fan_dst, double* __restrict__ out) {
  constexpr int R = kGroupiesBatch;
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= nb) return;
  const int64_t s = start[k], e = end[k];
  const double wk = width[k];
  const int u0 = blockIdx.y * rows_per, u1 = min(U, u0 + rows_per);
  for (int ub = u0; ub < u1; ub += R) {   // R source rows at a time: their loads in flight together
    const int nr = min(R, u1 - ub);
    const float* rows[R];
#pragma unroll
    for (int r = 0; r < R; ++r) rows[r] = x + row_off[ub + (r < nr ? r : 0)];
    float acc[R];
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] = 0.0f;
    if (e - s >= 2) {
      float a[R];
#pragma unroll
      for (int r = 0; r < R; ++r) a[r] = rows[r][s];
      int64_t i = s + 1;
      // four points of every row loaded before the ordered adds (each row's sequence unchanged)
      for (; i + 4 <= e; i += 4) {
        float b[R][4];
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
          for (int c = 0; c < 4; ++c) b[r][c] = rows[r][i + c];
#pragma unroll
        for (int r = 0; r < R; ++r) {
          acc[r] = (float)((double)acc[r] + (double)(a[r] + b[r][0]) / 2.0);
          acc[r] = (float)((double)acc[r] + (double)(b[r][0] + b[r][1]) / 2.0);
          acc[r] = (float)((double)acc[r] + (double)(b[r][1] + b[r][2]) / 2.0);
          acc[r] = (float)((double)acc[r] + (double)(b[r][2] + b[r][3]) / 2.0);
          a[r] = b[r][3];
        }
      }
      for (; i < e; ++i) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const float b = rows[r][i];
          acc[r] = (float)((double)acc[r] + (double)(a[r] + b) / 2.0);
          a[r] = b;
        }
      }
    }
    for (int r = 0; r < nr; ++r) {
      const double v = ((double)acc[r] * wk) * 1e-3;
      for (int f = fan_off[ub + r]; f < fan_off[ub + r + 1]; ++f)
        __builtin_nontemporal_store(v, out + fan_dst[f] + k);   // streaming: written once
    }
  }
}

// exact: one block per 256 output wavelengths and a range of source rows [u0, u1) (grid y).
// Per kExactBatch rows its lanes integrate the non-empty bins [glo, glo + ng) the block's
// interpolation brackets span into LDS ([kExactBatch][gcap], gcap the largest ng of the
// launch): xarray integrate (duck_array_ops.trapz), sum_i (dx_i * 0.5) * f64(f32(y_{i+1} + y_i))
// in point order, / (wl_max - wl_min) (opacity.py:40-42; a single-point bin gives 0 / 0 = NaN
// like the reference), four points' loads of four rows issued before their ordered adds.  One
// barrier, then every lane
// interpolates its wavelength, scipy interp1d(kind='linear', fill_value='extrapolate'):
// slope = (y_hi - y_lo) / (x_hi - x_lo), y = slope * (x - x_lo) + y_lo, and stores it to every
// destination row that selected the source row (the groupies fan-out), streaming.  HBM traffic:
// the selected source rows once (float32; a block boundary's bin is read by both blocks) and the
// destination table once (float64); no intermediate array.
constexpr int kExactBatch = 4;      // source rows integrated together (loads in flight)
constexpr int kExactCap = 160 * 1024 / (kExactBatch * 8);   // bins of one block's LDS window

// The integrals of bin [s, e) (width D) of nr <= R source rows: trapz in point order (above),
// four points' loads of every row in flight before their ordered adds.
template <int R>
__device__ __forceinline__ void bin_integrals(const float* const (&rows)[R], int64_t s, int64_t e,
                                              const double* __restrict__ hdx, double D,
                                              double (&out)[R]) {
  double acc[R];
  float prev[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    acc[r] = 0.0;
    prev[r] = rows[r][s];
  }
  int64_t i = s;
  for (; i + 4 < e; i += 4) {
    double h[4];
    float b[R][4];
#pragma unroll
    for (int c = 0; c < 4; ++c) h[c] = hdx[i + c];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int c = 0; c < 4; ++c) b[r][c] = rows[r][i + 1 + c];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        acc[r] = acc[r] + h[c] * (double)(b[r][c] + prev[r]);
        prev[r] = b[r][c];
      }
  }
  for (; i + 1 < e; ++i) {
    const double h = hdx[i];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const float b = rows[r][i + 1];
      acc[r] = acc[r] + h * (double)(b + prev[r]);
      prev[r] = b;
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r) out[r] = acc[r] / D;
}

// A block whose wavelengths' brackets span more than kExactCap bins (sparse wavelengths over a
// fine bin grid) has ng < 0: each lane integrates its own two bins (no LDS window, no barrier).
__global__ __launch_bounds__(256) void bin_exact_kernel(
    const float* __restrict__ x, const int64_t* __restrict__ row_off, int U, int rows_per,
    const int64_t* __restrict__ gstart, const int64_t* __restrict__ gend,
    const double* __restrict__ hdx, const double* __restrict__ Dx,
    const int32_t* __restrict__ blk_glo, const int32_t* __restrict__ blk_ng, int gcap,
    const int32_t* __restrict__ fan_off, const int64_t* __restrict__ fan_dst,
    const int32_t* __restrict__ lo, const double* __restrict__ xlo,
    const double* __restrict__ xhi, const double* __restrict__ lam, int64_t n,
    double* __restrict__ out) {
  constexpr int R = kExactBatch;
  extern __shared__ double integ[];   // [R][gcap]
  const int tid = threadIdx.x;
  const int64_t j = (int64_t)blockIdx.x * 256 + tid;
  const bool act = j < n;
  const int glo = blk_glo[blockIdx.x], ng = blk_ng[blockIdx.x];   // block-uniform
  const int32_t l = act ? lo[j] - glo : 0;
  const double dxj = act ? xhi[j] - xlo[j] : 1.0, tj = act ? lam[j] - xlo[j] : 0.0;
  const int u0 = blockIdx.y * rows_per, u1 = min(U, u0 + rows_per);
  for (int ub = u0; ub < u1; ub += R) {
    const int nr = min(R, u1 - ub);
    const float* rows[R];
#pragma unroll
    for (int r = 0; r < R; ++r) rows[r] = x + row_off[ub + (r < nr ? r : 0)];
    if (ng < 0) {   // per-lane brackets
      if (act) {
        const int g = glo + l;
        double ylo[R], yhi[R];
        bin_integrals<R>(rows, gstart[g], gend[g], hdx, Dx[g], ylo);
        bin_integrals<R>(rows, gstart[g + 1], gend[g + 1], hdx, Dx[g + 1], yhi);
        for (int r = 0; r < nr; ++r) {
          const double v = ((yhi[r] - ylo[r]) / dxj) * tj + ylo[r];
          for (int f = fan_off[ub + r]; f < fan_off[ub + r + 1]; ++f)
            __builtin_nontemporal_store(v, out + fan_dst[f] + j);
        }
      }
      continue;
    }
    for (int t = tid; t < ng; t += 256) {   // this lane's bins
      double v[R];
      bin_integrals<R>(rows, gstart[glo + t], gend[glo + t], hdx, Dx[glo + t], v);
#pragma unroll
      for (int r = 0; r < R; ++r) integ[r * gcap + t] = v[r];
    }
    __syncthreads();
    if (act) {
      for (int r = 0; r < nr; ++r) {
        const double ylo = integ[r * gcap + l], yhi = integ[r * gcap + l + 1];
        const double v = ((yhi - ylo) / dxj) * tj + ylo;
        for (int f = fan_off[ub + r]; f < fan_off[ub + r + 1]; ++f)
          __builtin_nontemporal_store(v, out + fan_dst[f] + j);
      }
    }
    __syncthreads();   // the next rows' integrals overwrite these
  }
}

// Synthetic DACE-like line forest for benchmarks (no host copy of n_T*n_p*n_hi values):
// 10^(-1.5 + 0.9 sin(1.7 ln wl) + 3 u^8) * (T / 1000)^0.5 * p^0.05, u = hash(i, seed).
__global__ void gen_xsec_kernel(float* __restrict__ x, int nT, int np, int64_t nhi,
                                const double* __restrict__ T, const double* __restrict__ p,
                                const double* __restrict__ wl, uint64_t seed) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nhi) return;
  uint64_t h = (uint64_t)i * 0x9E3779B97F4A7C15ull ^ seed;
  h ^= h >> 33;
  h *= 0xff51afd7ed558ccdull;
  h ^= h >> 33;
  const double u = (double)(h >> 11) * (1.0 / 9007199254740992.0);
  const double u2 = u * u, u4 = u2 * u2;
  const double base = pow(10.0, -1.5 + 0.9 * sin(1.7 * log(wl[i])) + 3.0 * u4 * u4);
  for (int a = 0; a < nT; ++a)
    for (int b = 0; b < np; ++b)
      x[((int64_t)a * np + b) * nhi + i] =
          (float)(base * sqrt(T[a] / 1000.0) * pow(p[b], 0.05));
}

// ------------------------------------------------------------------- host plan
// scipy interp1d 'nearest' after xarray sortby: midpoints x[i]/2 + x[i+1]/2, searchsorted
// side='left', clipped (opacity.py:26-29 interp_kwargs, fill_value='extrapolate').
std::vector<int> nearest_index(const std::vector<double>& nodes, const double* t, int n) {
  std::vector<int> order(nodes.size());
  std::iota(order.begin(), order.end(), 0);
  std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return nodes[a] < nodes[b]; });
  std::vector<double> bds;
  for (size_t i = 0; i + 1 < order.size(); ++i)
    bds.push_back(nodes[order[i + 1]] / 2.0 + nodes[order[i]] / 2.0);
  std::vector<int> out(n);
  for (int j = 0; j < n; ++j) {
    const int64_t k = std::lower_bound(bds.begin(), bds.end(), t[j]) - bds.begin();
    out[j] = order[std::min<int64_t>(k, (int64_t)order.size() - 1)];
  }
  return out;
}

// numpy pairwise summation (np.mean of the group wavelengths, opacity.py:42).
double pairwise_sum(const double* a, int64_t n) {
  if (n < 8) {
    double r = 0.0;
    for (int64_t i = 0; i < n; ++i) r += a[i];
    return r;
  }
  if (n <= 128) {
    double r[8];
    for (int j = 0; j < 8; ++j) r[j] = a[j];
    int64_t i = 8;
    for (; i < n - (n % 8); i += 8)
      for (int j = 0; j < 8; ++j) r[j] += a[i + j];
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; ++i) res += a[i];
    return res;
  }
  int64_t n2 = n / 2;
  n2 -= n2 % 8;
  return pairwise_sum(a, n2) + pairwise_sum(a + n2, n - n2);
}

struct Dest {
  // destination rows: (p index kp, T index kt) -> element offset in the output
  int n_p = 0, n_T = 0;
  std::vector<int64_t> off;  // [n_p * n_T] row-major over (kp, kt)
};

int check_ascending(const double* a, int64_t n, const char* what) {
  for (int64_t i = 0; i + 1 < n; ++i)
    if (!(a[i + 1] > a[i])) return set_error(std::string(what) + " must be strictly ascending");
  return 0;
}

// The whole binning of one species into device buffer `out` (rows at dest.off).
int bin_into(frei_xsec* x, int mode, const double* wl_bins, const double* lam, int64_t n_bins,
             int64_t lam_lo, int64_t n_out, const double* T_t, const double* p_t,
             const Dest& dest, double* d_out) {
  if (mode != FREI_BIN_GROUPIES && mode != FREI_BIN_EXACT) return set_error("unknown binning mode");
  if (n_bins < 1 || lam_lo < 0 || n_out < 1 || lam_lo + n_out > n_bins)
    return set_error("wavelength slice outside the grid");
  TRY(check_ascending(wl_bins, n_bins + 1, "wl_bins"));
  hipStream_t st = x->stream;
  const std::vector<double>& wl = x->wl;
  // pandas.cut(right=True) ranges on the cropped axis b_0 < x < b_last
  std::vector<int64_t> start(n_bins), end(n_bins);
  for (int64_t k = 0; k < n_bins; ++k) {
    start[k] = std::upper_bound(wl.begin(), wl.end(), wl_bins[k]) - wl.begin();
    end[k] = (k + 1 < n_bins ? std::upper_bound(wl.begin(), wl.end(), wl_bins[k + 1])
                             : std::lower_bound(wl.begin(), wl.end(), wl_bins[k + 1])) -
             wl.begin();
    end[k] = std::max(end[k], start[k]);
  }
  // nearest source nodes and the unique source rows they select
  const std::vector<int> ti = nearest_index(x->T, T_t, dest.n_T);
  const std::vector<int> pi = nearest_index(x->p, p_t, dest.n_p);
  std::map<int64_t, int> uid;  // source row -> unique index (ascending source order)
  for (int kp = 0; kp < dest.n_p; ++kp)
    for (int kt = 0; kt < dest.n_T; ++kt) uid[(int64_t)ti[kt] * x->np + pi[kp]] = 0;
  std::vector<int64_t> row_off;
  for (auto& kv : uid) {
    kv.second = (int)row_off.size();
    row_off.push_back(kv.first * x->nhi);
  }
  const int U = (int)row_off.size();
  std::vector<int32_t> dst_src(dest.off.size());
  for (int kp = 0; kp < dest.n_p; ++kp)
    for (int kt = 0; kt < dest.n_T; ++kt)
      dst_src[(size_t)kp * dest.n_T + kt] = uid[(int64_t)ti[kt] * x->np + pi[kp]];

  // fan-out: destination rows of every unique source row (CSR)
  std::vector<int32_t> fan_off(U + 1, 0);
  for (int32_t q : dst_src) fan_off[q + 1]++;
  for (int u = 0; u < U; ++u) fan_off[u + 1] += fan_off[u];
  std::vector<int64_t> fan_dst(dst_src.size());
  {
    std::vector<int32_t> fill(fan_off.begin(), fan_off.end() - 1);
    for (size_t d = 0; d < dst_src.size(); ++d) fan_dst[fill[dst_src[d]]++] = dest.off[d];
  }

  // (the host vectors outlive every copy: the stream is synchronised before returning, on every
  // path once a plan copy may be in flight, so the next call's stage_reserve never frees or
  // overwrites the pinned buffer under a running DMA; the timing events are destroyed there too)
  hipEvent_t ev[2] = {nullptr, nullptr};
  auto cleanup = [&]() {
    (void)hipStreamSynchronize(st);
    for (auto& e : ev)
      if (e) (void)hipEventDestroy(e), e = nullptr;
  };
  // every plan array of either mode (groups <= bins), with the 256-byte alignment of each
  const size_t plan_bytes = 4096 + 16 * ((size_t)U + 1) + 8 * fan_dst.size() +
                            24 * ((size_t)n_bins + 1) + 32 * (size_t)n_out +
                            8 * ((size_t)n_out / 256 + 1);
  if (int rc = stage_reserve(x, plan_bytes)) return rc;
  int64_t* d_row = nullptr;
  if (int rc = stage(x, 0, &d_row, row_off, st)) return cleanup(), rc;
  if (x->timing)
    for (auto& e : ev)
      if (hipEventCreate(&e) != hipSuccess) return cleanup(), set_error("hipEventCreate failed");
  int rc = 0;
  if (mode == FREI_BIN_GROUPIES) {
    // bins [lam_lo, lam_lo + n_out) map 1:1 to output wavelengths
    std::vector<int64_t> s(start.begin() + lam_lo, start.begin() + lam_lo + n_out),
        e(end.begin() + lam_lo, end.begin() + lam_lo + n_out);
    std::vector<double> w(n_out);
    for (int64_t k = 0; k < n_out; ++k) w[k] = wl_bins[lam_lo + k + 1] - wl_bins[lam_lo + k];
    int64_t *d_s = nullptr, *d_e = nullptr, *d_fd = nullptr;
    double* d_w = nullptr;
    int32_t* d_fo = nullptr;
    if ((rc = stage(x, 1, &d_s, s, st)) || (rc = stage(x, 2, &d_e, e, st)) ||
        (rc = stage(x, 3, &d_w, w, st)) || (rc = stage(x, 4, &d_fo, fan_off, st)) ||
        (rc = stage(x, 5, &d_fd, fan_dst, st)))
      return cleanup(), rc;
    const int rows_per = std::min(U, kGroupiesRows);
    dim3 grid((unsigned)((n_out + 255) / 256), (unsigned)((U + rows_per - 1) / rows_per));
    // timed: the plan uploads (pageable copies) complete first, so the events hold the kernel
    if (x->timing && (hipStreamSynchronize(st) != hipSuccess ||
                      hipEventRecord(ev[0], st) != hipSuccess))
      return cleanup(), set_error("binning: timing event failed");
    bin_groupies_kernel<<<grid, 256, 0, st>>>(x->d_x, d_row, U, rows_per, d_s, d_e, d_w, n_out,
                                              d_fo, d_fd, d_out);
  } else {
    // non-empty groups (xarray groupby_bins drops empty bins) and their coordinates
    std::vector<int64_t> gs, ge;
    std::vector<double> xc, Dx;
    for (int64_t k = 0; k < n_bins; ++k)
      if (end[k] > start[k]) {
        gs.push_back(start[k]);
        ge.push_back(end[k]);
        xc.push_back(pairwise_sum(wl.data() + start[k], end[k] - start[k]) /
                     (double)(end[k] - start[k]));
        Dx.push_back(wl[end[k] - 1] - wl[start[k]]);
      }
    const int64_t Gall = (int64_t)xc.size();
    if (Gall < 2) return cleanup(), set_error("x and y arrays must have at least 2 entries");
    // interval of each output wavelength: clip(searchsorted(x, lam), 1, G - 1)
    std::vector<int64_t> hi(n_out);
    for (int64_t j = 0; j < n_out; ++j) {
      const int64_t h = std::lower_bound(xc.begin(), xc.end(), lam[lam_lo + j]) - xc.begin();
      hi[j] = std::min<int64_t>(std::max<int64_t>(h, 1), Gall - 1);
    }
    const int64_t g0 = *std::min_element(hi.begin(), hi.end()) - 1;
    const int64_t g1 = *std::max_element(hi.begin(), hi.end()) + 1;  // groups [g0, g1)
    std::vector<int64_t> s(gs.begin() + g0, gs.begin() + g1), e(ge.begin() + g0, ge.begin() + g1);
    std::vector<double> dx(Dx.begin() + g0, Dx.begin() + g1);
    std::vector<int32_t> lo(n_out);
    std::vector<double> xlo(n_out), xhi(n_out), lamv(lam + lam_lo, lam + lam_lo + n_out);
    for (int64_t j = 0; j < n_out; ++j) {
      lo[j] = (int32_t)(hi[j] - 1 - g0);
      xlo[j] = xc[hi[j] - 1];
      xhi[j] = xc[hi[j]];
    }
    // per block of 256 output wavelengths: the bins its brackets span, from the smallest to
    // the largest lo of its lanes (any order of lam: scipy's interp1d takes unsorted x_new) —
    // about 257 when the wavelengths are the bin centres; a block spanning more than kExactCap
    // bins interpolates lane by lane (bng < 0)
    const int64_t nblk = (n_out + 255) / 256;
    std::vector<int32_t> bglo(nblk), bng(nblk);
    int gcap = 1;
    for (int64_t q = 0; q < nblk; ++q) {
      const int64_t ja = q * 256, jb = std::min(n_out, ja + 256);
      const auto mm = std::minmax_element(lo.begin() + ja, lo.begin() + jb);
      bglo[q] = *mm.first;
      const int64_t span = (int64_t)*mm.second + 2 - *mm.first;
      if (span > kExactCap) {
        bglo[q] = 0;   // lanes index the groups directly
        bng[q] = -1;
      } else {
        bng[q] = (int32_t)span;
        gcap = std::max(gcap, (int)span);
      }
    }
    const size_t lds = (size_t)kExactBatch * gcap * sizeof(double);
    if (lds > 64 * 1024 &&
        hipFuncSetAttribute(reinterpret_cast<const void*>(&bin_exact_kernel),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
      return cleanup(), set_error("binning: LDS opt-in failed");
    if (!x->d_hdx) {
      std::vector<double> h(std::max<int64_t>(x->nhi - 1, 1));
      for (int64_t i = 0; i + 1 < x->nhi; ++i) h[i] = (wl[i + 1] - wl[i]) * 0.5;
      if ((rc = upload(&x->d_hdx, h, st))) return cleanup(), rc;
    }
    int64_t *d_s = nullptr, *d_e = nullptr, *d_do = nullptr;
    double *d_D = nullptr, *d_xlo = nullptr, *d_xhi = nullptr, *d_lam = nullptr;
    int32_t *d_lo = nullptr, *d_fo = nullptr, *d_bglo = nullptr, *d_bng = nullptr;
    if ((rc = stage(x, 1, &d_s, s, st)) || (rc = stage(x, 2, &d_e, e, st)) ||
        (rc = stage(x, 3, &d_D, dx, st)) || (rc = stage(x, 4, &d_fo, fan_off, st)) ||
        (rc = stage(x, 5, &d_do, fan_dst, st)) || (rc = stage(x, 6, &d_lo, lo, st)) ||
        (rc = stage(x, 7, &d_xlo, xlo, st)) || (rc = stage(x, 8, &d_xhi, xhi, st)) ||
        (rc = stage(x, 9, &d_lam, lamv, st)) || (rc = stage(x, 10, &d_bglo, bglo, st)) ||
        (rc = stage(x, 11, &d_bng, bng, st)))
      return cleanup(), rc;
    // timed: the plan uploads (pageable copies) complete first, so the events hold the kernel
    if (x->timing && (hipStreamSynchronize(st) != hipSuccess ||
                      hipEventRecord(ev[0], st) != hipSuccess))
      return cleanup(), set_error("binning: timing event failed");
    const int rows_per = std::min(U, kExactRows);
    dim3 grid((unsigned)nblk, (unsigned)((U + rows_per - 1) / rows_per));
    bin_exact_kernel<<<grid, 256, lds, st>>>(x->d_x, d_row, U, rows_per, d_s, d_e, x->d_hdx,
                                             d_D, d_bglo, d_bng, gcap, d_fo, d_do, d_lo, d_xlo, d_xhi, d_lam,
                                           n_out, d_out);
  }
  if (hipGetLastError() != hipSuccess) return cleanup(), set_error("binning kernel launch failed");
  if (x->timing) {
    float ms = 0;
    if (hipEventRecord(ev[1], st) != hipSuccess || hipEventSynchronize(ev[1]) != hipSuccess ||
        hipEventElapsedTime(&ms, ev[0], ev[1]) != hipSuccess)
      return cleanup(), set_error("binning: timing event failed");
    x->t_ms += ms;
    x->t_n += 1;
  }
  if (hipStreamSynchronize(st) != hipSuccess) return cleanup(), set_error("binning kernels failed");
  cleanup();
  return 0;
}

}  // namespace

namespace frei {
// frei_set_table_binned (frei_runtime.hip): bin species into a context table whose rows for
// destination node (kp, kt) start at row_off[kp * n_T + kt].
int bin_into_table(frei_xsec* x, int mode, const double* wl_bins, const double* lam,
                   int64_t n_bins, int64_t lam_lo, int64_t n_out, const double* T_t, int n_T,
                   const double* p_t, int n_p, const int64_t* row_off, double* d_tab,
                   int device) {
  if (!x) return set_error("null cross-section");
  if (x->device != device) return set_error("cross-section and context are on different devices");
  Dest d;
  d.n_p = n_p;
  d.n_T = n_T;
  d.off.assign(row_off, row_off + (size_t)n_p * n_T);
  HIP_TRY(hipSetDevice(x->device));
  return bin_into(x, mode, wl_bins, lam, n_bins, lam_lo, n_out, T_t, p_t, d, d_tab);
}
}  // namespace frei

// ==================================================================== C ABI
extern "C" {

static int xsec_alloc(frei_xsec** out, int device, int n_T, int n_p, int64_t n_hi,
                      const double* T_nodes, const double* p_nodes, const double* wl_hi) {
  if (!out || !T_nodes || !p_nodes || !wl_hi) return set_error("null argument");
  *out = nullptr;
  if (n_T < 1 || n_p < 1 || n_hi < 2) return set_error("empty cross-section grid");
  TRY(check_ascending(wl_hi, n_hi, "high-resolution wavelengths"));
  frei_xsec* x = new frei_xsec();
  x->device = device;
  x->nT = n_T;
  x->np = n_p;
  x->nhi = n_hi;
  x->T.assign(T_nodes, T_nodes + n_T);
  x->p.assign(p_nodes, p_nodes + n_p);
  x->wl.assign(wl_hi, wl_hi + n_hi);
  if (hipSetDevice(device) != hipSuccess ||
      hipStreamCreateWithFlags(&x->stream, hipStreamNonBlocking) != hipSuccess ||
      hipMalloc((void**)&x->d_x, (size_t)n_T * n_p * n_hi * sizeof(float)) != hipSuccess) {
    frei_xsec_destroy(x);
    return set_error("frei_xsec: device allocation failed");
  }
  *out = x;
  return 0;
}

int frei_xsec_create(frei_xsec** out, int device, const float* values, int n_T, int n_p,
                     int64_t n_hi, const double* T_nodes, const double* p_nodes,
                     const double* wl_hi) {
  if (!values) return set_error("null argument");
  TRY(xsec_alloc(out, device, n_T, n_p, n_hi, T_nodes, p_nodes, wl_hi));
  frei_xsec* x = *out;
  if (hipMemcpy(x->d_x, values, (size_t)n_T * n_p * n_hi * sizeof(float),
                hipMemcpyHostToDevice) != hipSuccess) {
    frei_xsec_destroy(x);
    *out = nullptr;
    return set_error("frei_xsec_create: host-to-device copy failed");
  }
  return 0;
}

int frei_xsec_create_synthetic(frei_xsec** out, int device, int n_T, int n_p, int64_t n_hi,
                               const double* T_nodes, const double* p_nodes,
                               const double* wl_hi, uint64_t seed) {
  TRY(xsec_alloc(out, device, n_T, n_p, n_hi, T_nodes, p_nodes, wl_hi));
  frei_xsec* x = *out;
  double *d_T = nullptr, *d_p = nullptr, *d_wl = nullptr;
  int rc = 0;
  if ((rc = upload(&d_T, x->T, x->stream)) || (rc = upload(&d_p, x->p, x->stream)) ||
      (rc = upload(&d_wl, x->wl, x->stream))) {
    dfree(d_T), dfree(d_p), dfree(d_wl);
    frei_xsec_destroy(x);
    *out = nullptr;
    return rc;
  }
  gen_xsec_kernel<<<(unsigned)((n_hi + 255) / 256), 256, 0, x->stream>>>(x->d_x, n_T, n_p, n_hi,
                                                                        d_T, d_p, d_wl, seed);
  const bool ok = hipGetLastError() == hipSuccess && hipStreamSynchronize(x->stream) == hipSuccess;
  dfree(d_T), dfree(d_p), dfree(d_wl);
  if (!ok) {
    frei_xsec_destroy(x);
    *out = nullptr;
    return set_error("frei_xsec_create_synthetic: generation failed");
  }
  return 0;
}

int frei_xsec_destroy(frei_xsec* x) {
  if (!x) return 0;
  (void)hipSetDevice(x->device);
  if (x->stream) (void)hipStreamSynchronize(x->stream);
  dfree(x->d_x);
  dfree(x->d_hdx);
  dfree(x->d_scratch);
  for (auto& b : x->plan)
    if (b.first) (void)hipFree(b.first);
  if (x->pinned) (void)hipHostFree(x->pinned);
  if (x->stream) (void)hipStreamDestroy(x->stream);
  delete x;
  return 0;
}

int frei_xsec_bin(frei_xsec* x, int mode, const double* wl_bins, const double* lam,
                  int64_t n_bins, const double* T_nodes, int n_T, const double* p_nodes,
                  int n_p, double* out) {
  if (!x || !wl_bins || !lam || !T_nodes || !p_nodes) return set_error("null argument");
  if (n_T < 1 || n_p < 1) return set_error("need at least one target (T, p) node");
  HIP_TRY(hipSetDevice(x->device));
  const size_t total = (size_t)n_p * n_T * n_bins;
  if (x->scratch_n < total) {
    dfree(x->d_scratch);
    x->scratch_n = 0;
    TRY(dalloc(&x->d_scratch, total));
    x->scratch_n = total;
  }
  Dest d;
  d.n_p = n_p;
  d.n_T = n_T;
  d.off.resize((size_t)n_p * n_T);
  for (size_t r = 0; r < d.off.size(); ++r) d.off[r] = (int64_t)r * n_bins;
  TRY(bin_into(x, mode, wl_bins, lam, n_bins, 0, n_bins, T_nodes, p_nodes, d, x->d_scratch));
  if (out) HIP_TRY(hipMemcpy(out, x->d_scratch, total * sizeof(double), hipMemcpyDeviceToHost));
  return 0;
}

int frei_xsec_timing(frei_xsec* x, int on, double* total_ms, int* n_calls) {
  if (!x) return set_error("null argument");
  if (total_ms) *total_ms = x->t_ms;
  if (n_calls) *n_calls = x->t_n;
  if (on >= 0) {
    x->timing = on != 0;
    x->t_ms = 0;
    x->t_n = 0;
  }
  return 0;
}

}  // extern "C"
