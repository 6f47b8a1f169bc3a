// Shared device-side building blocks for the gfx950 KFAC kernels.
//
// The fp32 contraction core stages 32-row x 64-column panels of two operands
// through LDS (register staging, double-buffered, one barrier per stage) and
// accumulates a 64x64 output tile with v_mfma_f32_32x32x2_f32 (exact fp32
// products, k-ordered fma chain): 4 waves, one 32x32 quadrant each.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/kfac_hip.h"
#include "knobs.h"

namespace kfac {

constexpr int TILE = 64;        // output tile edge
constexpr int BK = 32;          // rows of k staged per pipeline step
constexpr int LDP = TILE + 1;   // padded LDS row pitch (floats): column writes conflict-free
constexpr int NTHREADS = 256;   // 4 waves
constexpr int PANEL = BK * (TILE + 4); // floats per staged panel (max pitch)

typedef float floatx16 __attribute__((ext_vector_type(16)));

#define KFAC_CHECK_LAUNCH()                                   \
  do {                                                        \
    if (hipGetLastError() != hipSuccess) return KFAC_ELAUNCH; \
  } while (0)

static inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }
static inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// ---- optional launch timing (capi.hip): Prof scope records hipEvents around a launch
// `work` / `bytes`: the launch's algorithmic flops and HBM bytes (factor kernels: sum
// over jobs of K rows x n (n + 1), and of the operand's bytes read once), summed per
// slot by kfac_profile_read_work so a roofline names its own kernel's work
bool prof_on();
void prof_begin(int id, hipStream_t s, double work = 0.0, double bytes = 0.0);
void prof_end(int id, hipStream_t s);
struct ProfScope {
  int id;
  hipStream_t s;
  ProfScope(int id_, hipStream_t s_, double work = 0.0, double bytes = 0.0) : id(id_), s(s_) {
    prof_begin(id, s, work, bytes);
  }
  ~ProfScope() { prof_end(id, s); }
};

// Device copy of kfac_operand with the derived ones-column index.
struct OpDev {
  const float* ptr;
  int64_t rows;
  int64_t last_rows;  // multi-batch ROWMAJOR job: rows of the ragged last batch (0: rows)
  int64_t ld, L, sB;
  int32_t layout, cols, ones;  // ones = cols if has_ones else -1
  int32_t C, H, W, kh, kw, sh, sw, ph, pw, Ho, Wo;
};

static inline OpDev to_dev(const kfac_operand& o) {
  OpDev d;
  d.ptr = o.ptr;
  d.rows = o.rows;
  d.last_rows = o.last_rows;
  d.ld = o.ld;
  d.L = o.L;
  d.sB = o.sB;
  d.layout = o.layout;
  d.cols = o.cols;
  d.ones = o.has_ones ? o.cols : -1;
  d.C = o.C; d.H = o.H; d.W = o.W; d.kh = o.kh; d.kw = o.kw;
  d.sh = o.sh; d.sw = o.sw; d.ph = o.ph; d.pw = o.pw; d.Ho = o.Ho; d.Wo = o.Wo;
  return d;
}

// ---------------------------------------------------------------- panel loaders
// Each thread owns 8 elements of a 32 x 64 panel.  ROWMAJOR walks columns with
// the lanes (coalesced along a row); CHANNEL/PATCH walk rows with the lanes
// (coalesced along the contiguous spatial index).
template <int LAYOUT>
struct Panel;

// ROWMAJOR: 16-byte loads (16 lanes cover one 256-byte panel row) and
// ds_write_b128 into a [k][i] image with a 16-byte-aligned pitch; columns at the
// right edge (ones column, ragged widths, unaligned rows) fall back to scalars.
template <>
struct Panel<KFAC_ROWMAJOR> {
  static constexpr int PITCH = TILE + 4;
  const float* base;
  int64_t ld, kend;
  int col, c4, r0, cols, ones;
  bool vec;
  __device__ __forceinline__ void init(const OpDev& op, const float* base_, int col0, int tid,
                                       int64_t k_end, int64_t) {
    base = base_; ld = op.ld; kend = k_end; cols = op.cols; ones = op.ones;
    c4 = (tid & 15) * 4; r0 = tid >> 4; col = col0 + c4;
    vec = (col + 3 < cols) && ((ld & 3) == 0) && ((reinterpret_cast<uintptr_t>(base) & 15) == 0);
  }
  __device__ __forceinline__ void load(int64_t k, float (&v)[8]) const {
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      const int64_t row = k + r0 + 16 * m;
      float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
      if (row < kend) {
        const float* p = base + row * ld + col;
        if (vec) {
          x = *reinterpret_cast<const float4*>(p);
        } else {
          float e[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int cq = col + q;
            e[q] = cq < cols ? p[q] : (cq == ones ? 1.f : 0.f);
          }
          x = make_float4(e[0], e[1], e[2], e[3]);
        }
      }
      v[4 * m + 0] = x.x; v[4 * m + 1] = x.y; v[4 * m + 2] = x.z; v[4 * m + 3] = x.w;
    }
  }
  __device__ __forceinline__ void store(float* lds, const float (&v)[8]) const {
#pragma unroll
    for (int m = 0; m < 2; ++m)
      *reinterpret_cast<float4*>(lds + (r0 + 16 * m) * PITCH + c4) =
          make_float4(v[4 * m], v[4 * m + 1], v[4 * m + 2], v[4 * m + 3]);
  }
};

// CHANNEL and PATCH walk the K rows (image b, position l) incrementally: loads are
// issued for k_first, k_first + BK, ... in order, so one division at init replaces
// a 64-bit division per stage.
template <>
struct Panel<KFAC_CHANNEL> {
  static constexpr int PITCH = LDP;
  const float* base;
  int64_t L, sB, kend, b, l;  // (b, l) of row k + r for the next load
  int r, c0, col0, cols, ones;
  __device__ __forceinline__ void init(const OpDev& op, const float* base_, int col0_, int tid,
                                       int64_t k_end, int64_t k_first) {
    base = base_; L = op.L; sB = op.sB; kend = k_end; cols = op.cols; ones = op.ones;
    r = tid & 31; c0 = tid >> 5; col0 = col0_;
    const int64_t row = k_first + r;
    b = row / L;
    l = row - b * L;
  }
  __device__ __forceinline__ void load(int64_t k, float (&v)[8]) {
    const bool ok = k + r < kend;
    const int64_t off = b * sB + l;
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const int col = col0 + c0 + 8 * m;
      float x = 0.f;
      if (ok) x = col < cols ? base[off + (int64_t)col * L] : (col == ones ? 1.f : 0.f);
      v[m] = x;
    }
    l += BK;
    while (l >= L) { l -= L; ++b; }
  }
  __device__ __forceinline__ void store(float* lds, const float (&v)[8]) const {
#pragma unroll
    for (int m = 0; m < 8; ++m) lds[r * LDP + c0 + 8 * m] = v[m];
  }
};

template <>
struct Panel<KFAC_PATCH> {
  static constexpr int PITCH = LDP;
  static constexpr int KZERO = -1, KONES = -2;
  const float* base;
  int64_t sB, kend, b;  // image of row k + r for the next load
  int r, c0, H, W, Ho, Wo, sh, sw, ph, pw, oh, ow;
  int coff[8];
  int kij[8];  // (ki << 16) | kj, or KZERO / KONES
  __device__ __forceinline__ void init(const OpDev& op, const float* base_, int col0, int tid,
                                       int64_t k_end, int64_t k_first) {
    base = base_; sB = op.sB; kend = k_end;
    H = op.H; W = op.W; Ho = op.Ho; Wo = op.Wo; sh = op.sh; sw = op.sw; ph = op.ph; pw = op.pw;
    r = tid & 31; c0 = tid >> 5;
    const int64_t row = k_first + r;
    b = row / op.L;
    const int l = (int)(row - b * op.L);
    oh = l / Wo;
    ow = l - oh * Wo;
    const int kk = op.kh * op.kw;
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const int col = col0 + c0 + 8 * m;
      if (col < op.cols) {
        const int ch = col / kk, rem = col - ch * kk;
        const int ki = rem / op.kw, kj = rem - ki * op.kw;
        coff[m] = ch * H * W + ki * W + kj;
        kij[m] = (ki << 16) | kj;
      } else {
        coff[m] = 0;
        kij[m] = (col == op.ones) ? KONES : KZERO;
      }
    }
  }
  __device__ __forceinline__ void load(int64_t k, float (&v)[8]) {
    const bool ok = k + r < kend;
    const int ihb = oh * sh - ph, iwb = ow * sw - pw;
    const int64_t off = b * sB + (int64_t)ihb * W + iwb;
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      float x = 0.f;
      if (ok) {
        const int t = kij[m];
        if (t == KONES) {
          x = 1.f;
        } else if (t >= 0) {
          const int ih = ihb + (t >> 16), iw = iwb + (t & 0xffff);
          if ((unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W) x = base[off + coff[m]];
        }
      }
      v[m] = x;
    }
    ow += BK;
    while (ow >= Wo) {
      ow -= Wo;
      if (++oh == Ho) { oh = 0; ++b; }
    }
  }
  __device__ __forceinline__ void store(float* lds, const float (&v)[8]) const {
#pragma unroll
    for (int m = 0; m < 8; ++m) lds[r * LDP + c0 + 8 * m] = v[m];
  }
};

// ------------------------------------------------------------ contraction core
// acc(wave quadrant) += sum_{k in [k0,k1)} A[k][i0 + qi*32 + i] * B[k][j0 + qj*32 + j]
// lds: 2 buffers x 2 panels x PANEL floats.  `same` = B panel identical to A's.
// `active` = this wave's quadrant is needed (waves always join staging/barriers).
// `narrow`: only quadrant (0,0) is needed (factor edge <= 32): every wave computes
// it over its own quarter of each stage's K rows (the caller sums the 4 partials).
// `base` (null: opA.ptr / opB.ptr) replaces both operands' base pointer (one batch of
// a multi-batch job; then opA and opB are the same operand).
template <int LA, int LB>
__device__ __forceinline__ void contract_tile(const OpDev& opA, int i0, const OpDev& opB, int j0,
                                              int64_t k0, int64_t k1, bool same, bool active,
                                              float* lds, floatx16& acc, bool narrow = false,
                                              const float* base = nullptr) {
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int qi = narrow ? 0 : wave >> 1, qj = narrow ? 0 : wave & 1;
  const int h = lane >> 5, rr = lane & 31;

  Panel<LA> pa;
  Panel<LB> pb;
  pa.init(opA, base ? base : opA.ptr, i0, tid, k1, k0);
  pb.init(opB, base ? base : opB.ptr, j0, tid, k1, k0);
  float va[8], vb[8];

  // buffer c: A panel at lds + 2*c*PANEL, B panel right after it
  pa.load(k0, va);
  if (!same) pb.load(k0, vb);
  pa.store(lds, va);
  if (!same) pb.store(lds + PANEL, vb);
  __syncthreads();

  int cur = 0;
  for (int64_t k = k0; k < k1; k += BK) {
    const bool more = k + BK < k1;
    if (more) {
      pa.load(k + BK, va);
      if (!same) pb.load(k + BK, vb);
    }
    float* bcur = lds + 2 * cur * PANEL;
    const float* a = bcur + h * Panel<LA>::PITCH + qi * 32 + rr;
    const float* b = bcur + (same ? 0 : PANEL) + h * Panel<LB>::PITCH + qj * 32 + rr;
    if (narrow) {
#pragma unroll
      for (int s = 0; s < BK / 8; ++s) {
        const int ks = 2 * (wave * (BK / 8) + s);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[ks * Panel<LA>::PITCH], b[ks * Panel<LB>::PITCH],
                                                   acc, 0, 0, 0);
      }
    } else if (active) {
#pragma unroll
      for (int s = 0; s < BK / 2; ++s)
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[2 * s * Panel<LA>::PITCH],
                                                   b[2 * s * Panel<LB>::PITCH], acc, 0, 0, 0);
    }
    if (more) {
      float* bnext = lds + 2 * (cur ^ 1) * PANEL;
      pa.store(bnext, va);
      if (!same) pb.store(bnext + PANEL, vb);
    }
    __syncthreads();
    cur ^= 1;
  }
}

// Row within the wave's 32x32 quadrant held in accumulator register v of `lane`
// (v_mfma_f32_32x32x2_f32 C/D layout: col = lane & 31).
__device__ __forceinline__ int acc_row(int v, int lane) {
  return (v & 3) + 8 * (v >> 2) + 4 * (lane >> 5);
}

// Decode a lower-triangle tile index t -> (ti, tj), ti >= tj.
// Workgroups are dispatched round-robin over the 8 XCDs (block b -> XCD b % 8), each
// with its own 4 MB L2.  Hand every XCD a contiguous range of the logical task order
// so tasks that share operand rows share an L2.  Bijective for any n.
__device__ __forceinline__ int xcd_task(int b, int n) {
  const int x = b & 7, s = b >> 3, per = n >> 3, rem = n & 7;
  return (x < rem ? x * (per + 1) : rem * (per + 1) + (x - rem) * per) + s;
}

__device__ __forceinline__ void tri_decode(int t, int& ti, int& tj) {
  int i = (int)((sqrtf(8.f * (float)t + 1.f) - 1.f) * 0.5f);
  while ((i + 1) * (i + 2) / 2 <= t) ++i;
  while (i * (i + 1) / 2 > t) --i;
  ti = i;
  tj = t - i * (i + 1) / 2;
}

}  // namespace kfac
