// Kronecker-factor accumulation (KFAC.update) on gfx950.
//
// Replaces models/curvatures.py:341-363: per layer A = [a 1]^T[a 1]/cols and
// G = g^T g/cols (Conv2d through an implicit im2col / channel-major view instead
// of F.unfold + permute().contiguous() copies), then state = state + factor.
//
// One KFAC.update() = two launches for ALL layers' factors:
//   1. kfac_factor_tiles : grouped split-K fp32-MFMA SYRK.  A task is one
//      64x64 lower-triangle tile of one factor over one K-chunk; it writes a
//      64x64 fp32 partial slab (deterministic, no atomics).
//   2. kfac_factor_reduce: per tile, sum the slabs in split order, apply
//      F = beta*F + alpha*sum, write the tile and its mirror (LDS transpose),
//      so F stays exactly symmetric.
#include <algorithm>
#include <cstddef>
#include <array>
#include <functional>
#include <mutex>
#include <initializer_list>
#include <utility>
#include <vector>
#include <type_traits>

#include "kfac_common.h"

namespace kfac {

constexpr int MAXJ = 16;  // factor jobs per launch (kernarg budget: ~3.2 KB of 4 KB)
constexpr int KSEG = 64;  // batch base pointers per launch (multi-batch jobs; +512 B)

struct FactorJobDev {
  OpDev x;
  float alpha, beta;
  float* F;
  int64_t ldF;
  float* slab;       // this job's slabs: tiles*splits x 64 x 64
  int seg_off;       // multi-batch job: its batch bases are FactorArgs::segs[seg_off..] (else -1)
  int64_t chunk;     // BK-row stages per split
  int64_t nst;       // stages of the job: nseg * sps
  int sps, nseg;     // stages per batch (a stage never straddles two batches), batches
  int n, t, splits;  // factor edge, tiles per edge, K-splits
  int task_begin;    // first global task of this job
  int glds;          // row-major, 16-byte-aligned rows: LDS-DMA kernel
  int tile_begin;    // first global tile of this job (reduce launch)
  int accum;         // deferred reduction: `slab` is the caller's accumulator
  float sbeta;       // accumulator update: slab = sbeta*slab + alpha*partial
  int x3pair;        // kfac_factor_tiles_x3: thin last tile row, diagonal + edge tiles paired
  int sstride;       // slabs per tile of `slab` (a job's split s of tile t: t * sstride + s)
  int xsplits;       // x3 thin-row pairs: of the `splits` slabs per tile, the last xsplits are
                     // written by extra, shorter K-splits of the pair units only (x3_xsplits)
  // ragged last batch (x.last_rows, kfac_factor_tiles_x3 / narrow tasks only): its first
  // stage `rstage` (-1: none); its rows weigh rows / last_rows = `rw` times the others'
  // (its own per-batch mean): a task crossing into it scales its sums by 1 / rw = `rinv`
  // at rstage, and every task ending in it scales by rw at the end
  int64_t rstage;
  float rw, rinv;
  int rdelta;        // rows - last_rows (0: no ragged batch)
};

struct FactorArgs {
  const float* segs[KSEG];  // batch bases of the multi-batch jobs (kernel arguments: no copy)
  int njobs;
  int split_major;  // LDS-DMA path task order: 1 split-major, 0 tile-major (KFAC_SYRK_ORDER)
  int task_end[MAXJ];
  int tile_end[MAXJ];
  FactorJobDev job[MAXJ];
};

// Epilogue write of one lane's 16 partial-tile values (`at(v)` = address of value
// v): a plain slab store, or, for a deferred-reduction job, the accumulator update
// slab = sbeta*slab + alpha*partial (old values loaded together first).
template <class At>
__device__ __forceinline__ void put_partial(const FactorJobDev& J, const floatx16& acc, At at) {
  if (!J.accum) {
#pragma unroll
    for (int v = 0; v < 16; ++v) *at(v) = acc[v];
    return;
  }
  if (J.sbeta == 0.f) {
#pragma unroll
    for (int v = 0; v < 16; ++v) *at(v) = J.alpha * acc[v];
    return;
  }
  float old[16];
#pragma unroll
  for (int v = 0; v < 16; ++v) old[v] = *at(v);
#pragma unroll
  for (int v = 0; v < 16; ++v) *at(v) = fmaf(J.sbeta, old[v], J.alpha * acc[v]);
}

// The same for the first nb of a wave's N blocks (`at(i, v)`: value v of block i), split
// in two so the old values of every block are loaded before the first store (one round
// trip to the slab instead of nb: the compiler keeps a block's loads behind the previous
// block's stores) and can be in flight across the caller's partial-sum exchange.
template <int N, class At>
__device__ __forceinline__ void load_partials(const FactorJobDev& J, int nb, float (&old)[N][16], At at) {
  if (!J.accum || J.sbeta == 0.f) return;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    if (i >= nb) break;
#pragma unroll
    for (int v = 0; v < 16; ++v) old[i][v] = *at(i, v);
  }
}
template <int N, class At>
__device__ __forceinline__ void put_partials(const FactorJobDev& J, int nb, const floatx16 (&acc)[N],
                                             const float (&old)[N][16], At at) {
  const bool upd = J.accum && J.sbeta != 0.f;
  const float a = J.accum ? J.alpha : 1.f;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    if (i >= nb) break;
#pragma unroll
    for (int v = 0; v < 16; ++v) *at(i, v) = upd ? fmaf(J.sbeta, old[i][v], a * acc[i][v]) : a * acc[i][v];
  }
}

// K is walked in BK-row stages; stage s of a job is rows [k, k + BK) of batch
// `seg` (s = seg * sps + k / BK), so a multi-batch job reads each batch in place.
// `segs` = FactorArgs::segs (kernel-argument memory; never null: a conditional
// null pointer here makes the compiler copy the whole argument block to scratch).
__device__ __forceinline__ const float* seg_base(const FactorJobDev& J, const float* const* segs,
                                                 int seg) {
  return J.seg_off >= 0 ? segs[J.seg_off + seg] : J.x.ptr;
}

// rows of batch `seg` of a job (its ragged last batch: x.last_rows).  Arithmetic, not a
// select of two fields: a select of two argument-block addresses makes the compiler
// copy the whole FactorArgs to scratch (4.5 KB per lane)
__device__ __forceinline__ int64_t seg_rows(const FactorJobDev& J, int seg) {
  return J.x.rows - (int64_t)(seg == J.nseg - 1) * J.rdelta;
}

// the ragged last batch's weight on a task's partial sums (see FactorJobDev::rstage)
template <int NA>
__device__ __forceinline__ void scale_acc(floatx16 (&acc)[NA], float f) {
#pragma unroll
  for (int a = 0; a < NA; ++a)
#pragma unroll
    for (int v = 0; v < 16; ++v) acc[a][v] *= f;
}

struct StageCursor {
  int seg;
  int64_t k;  // first row of the stage within batch `seg`
  __device__ __forceinline__ void init(const FactorJobDev& J, int64_t s) {
    seg = (int)(s / J.sps);
    k = (s - (int64_t)seg * J.sps) * BK;
  }
  __device__ __forceinline__ void next(int64_t rows) {
    k += BK;
    if (k >= rows) { k = 0; ++seg; }
  }
};

// Narrow factors (n <= 32): the 4 waves hold partial sums of quadrant (0,0) over
// disjoint K subsets; sum them through LDS in wave order (deterministic) and store
// the quadrant.  `lds` is free (the caller's stage loop has ended with a barrier).
template <int NW = 4>
__device__ __forceinline__ void store_narrow(const FactorJobDev& J, float* out, floatx16& acc,
                                             float* lds) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __syncthreads();
  if (wave > 0) {
#pragma unroll
    for (int v = 0; v < 16; ++v) lds[((wave - 1) * 16 + v) * 64 + lane] = acc[v];
  }
  __syncthreads();
  if (wave != 0) return;
#pragma unroll
  for (int w = 0; w < NW - 1; ++w)
#pragma unroll
    for (int v = 0; v < 16; ++v) acc[v] += lds[(w * 16 + v) * 64 + lane];
  put_partial(J, acc, [&](int v) { return &out[acc_row(v, lane) * TILE + (lane & 31)]; });
}

template <int LAYOUT>
__device__ __forceinline__ void factor_task(const FactorJobDev& J, const float* const* segs, int local,
                                            float* lds) {
  // tile-major order: a tile's splits are consecutive tasks (one XCD; see the reduce)
  const int tile = local / J.splits, split = local - tile * J.splits;
  int ti, tj;
  tri_decode(tile, ti, tj);
  const int64_t s0 = (int64_t)split * J.chunk;
  const int64_t s1 = min(J.nst, s0 + J.chunk);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int qi = wave >> 1, qj = wave & 1;
  const bool diag = ti == tj;
  // strictly-upper quadrant of a diagonal tile, or a quadrant wholly in the tile
  // padding (rows or columns >= n): no MFMA work (the reduce never reads it)
  const bool active = !(diag && qi < qj) && ti * TILE + qi * 32 < J.n && tj * TILE + qj * 32 < J.n;
  floatx16 acc;
#pragma unroll
  for (int v = 0; v < 16; ++v) acc[v] = 0.f;
  const bool narrow = J.n <= 32;  // one 32x32 quadrant: the 4 waves split K instead
  if constexpr (LAYOUT == KFAC_ROWMAJOR) {
    // one pipelined contraction per batch piece of this split's stage range
    StageCursor c;
    c.init(J, s0);
    for (int64_t s = s0; s < s1;) {
      const int64_t here = min(s1 - s, (int64_t)J.sps - c.k / BK);
      contract_tile<LAYOUT, LAYOUT>(J.x, ti * TILE, J.x, tj * TILE, c.k,
                                    min(J.x.rows, c.k + here * BK), diag, active, lds, acc, narrow,
                                    seg_base(J, segs, c.seg));
      s += here;
      c.seg += 1;
      c.k = 0;
    }
  } else {
    // channel-major / im2col jobs are single-batch (validate()): stage s = rows [s*BK, ..)
    contract_tile<LAYOUT, LAYOUT>(J.x, ti * TILE, J.x, tj * TILE, s0 * BK, min(J.x.rows, s1 * BK),
                                  diag, active, lds, acc, narrow);
  }
  if (narrow) {
    store_narrow(J, J.slab + ((size_t)tile * J.sstride + split) * TILE * TILE, acc, lds);
    return;
  }
  if (!active) return;
  float* out = J.slab + ((size_t)tile * J.sstride + split) * TILE * TILE + qi * 32 * TILE + qj * 32;
  put_partial(J, acc, [&](int v) { return &out[acc_row(v, lane) * TILE + (lane & 31)]; });
}


// One block = one 16-row strip of one 64x64 tile: float4 slab reads (all splits
// in flight at once), F = beta*F + alpha*sum, then the mirrored strip through LDS.
// ---------------------------------------------------------------------------
// Row-major operands with 16-byte-aligned rows (cols, ld multiples of 4): panels
// arrive by LDS-DMA (global_load_lds_dwordx4) into a 3-slot ring, two stages in
// flight, counted vmcnt + raw s_barrier (one per stage), no staging VGPRs.  The
// image is lane-linear [32 rows][64 cols] (256-byte rows, unpadded: the MFMA's
// ds_read_b32 halves read 32 consecutive dwords, conflict-free).  Chunks past the
// last real column (bias ones column, tile padding) and rows past the range load
// from a safe address and are overwritten with their fill value once landed.
// GBK rows per stage; each thread of NW waves owns NCH = GBK/(4 NW) of a panel's
// 16-byte chunks.
template <int GBK, int NW = 4>
struct GldsPanel {
  static constexpr int NCH = GBK / (4 * NW);
  // chunk i of wave w, lane l: row (w NCH + i) * 4 + (l >> 4), columns col .. col + 3
  // with col = col0 + 4 (l & 15) -- the same columns for every chunk of the lane
  int64_t ld, kend;
  int col, ones, lrow;
  bool real;   // the lane's chunks hold matrix data (else fill: ones column -> 1)
  bool fillw;  // some lane of the wave has fill chunks
  __device__ __forceinline__ void init(const OpDev& op, int col0, int w, int lane, int64_t k_end) {
    ld = op.ld; kend = k_end;
    col = col0 + (lane & 15) * 4;
    real = col < op.cols;
    ones = op.ones;
    lrow = w * NCH * 4 + (lane >> 4);
    fillw = __ballot(!real) != 0;
  }
  // issue the LDS-DMA loads of rows [k, k+GBK) of the batch at `base` into `slot`
  __device__ __forceinline__ void issue(const float* base, int64_t k, float* slot, int w) const {
    if (k + GBK <= kend) {  // whole stage inside the batch: no row clamp
      const float* p = base + (k + lrow) * ld + (real ? col : 0);
#pragma unroll
      for (int i = 0; i < NCH; ++i)
        __builtin_amdgcn_global_load_lds(p + 4 * i * ld, slot + (w * NCH + i) * 256, 16, 0, 0);
      return;
    }
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int64_t row = k + lrow + 4 * i;
      const int64_t r = row < kend ? row : kend - 1;
      const float* src = base + r * ld + (real ? col : 0);
      __builtin_amdgcn_global_load_lds(src, slot + (w * NCH + i) * 256, 16, 0, 0);
    }
  }
  // after landing: overwrite chunks that must not hold matrix data (none: a whole
  // stage of real columns)
  __device__ __forceinline__ void fixup(int64_t k, float* slot) const {
    if (!fillw && k + GBK <= kend) return;
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const bool okrow = k + lrow + 4 * i < kend;
      if (!real || !okrow) {
        // inline asm: the explicit vm_wait already covers this lane's DMA; a plain
        // store would make the compiler drain every in-flight stage (vmcnt(0))
        typedef float f4v __attribute__((ext_vector_type(4)));
        f4v v = {0.f, 0.f, 0.f, 0.f};
        if (okrow) {
#pragma unroll
          for (int q = 0; q < 4; ++q) v[q] = col + q == ones ? 1.f : 0.f;
        }
        const uint32_t addr = (uint32_t)(uintptr_t)(slot + ((lrow / 4 + i) * 64 + lane) * 4);
        asm volatile("ds_write_b128 %0, %1" ::"v"(addr), "v"(v) : "memory");
      }
    }
  }
};

__device__ __forceinline__ void vm_wait(int n) {
  // counted waits need immediates: n = DMA instructions allowed to stay in flight
  switch (n) {
    case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 9: asm volatile("s_waitcnt vmcnt(9)" ::: "memory"); break;
    case 12: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
    case 18: asm volatile("s_waitcnt vmcnt(18)" ::: "memory"); break;
    case 24: asm volatile("s_waitcnt vmcnt(24)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

__device__ __forceinline__ void stage_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
}

// Narrow row-major factors (n <= 32) whose rows are not 16-B aligned (the MLP's
// 10-wide output gradient): operands go from global memory straight into the MFMA
// registers, one stage ahead, so the glds-only launch (32 KB of LDS) takes them
// too.  Of NW waves, wave w takes rows (BK/NW) w .. of every 32-row stage (the waves
// split K; the store sums them), lane (rr, h) row 2*s2 + h, column rr (the ones
// column: 1).
template <int NW = 4>
__device__ __forceinline__ void narrow_direct_load(const FactorJobDev& J, const float* base, int64_t k0,
                                                   int64_t rows, float (&v)[BK / (2 * NW)]) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, rr = lane & 31, h = lane >> 5;
#pragma unroll
  for (int s2 = 0; s2 < BK / (2 * NW); ++s2) {
    const int64_t k = k0 + 2 * (wave * (BK / (2 * NW)) + s2) + h;
    v[s2] = k < rows ? (rr < J.x.cols ? base[k * J.x.ld + rr] : (rr == J.x.ones ? 1.f : 0.f)) : 0.f;
  }
}

template <int NW = 4>
__device__ __forceinline__ void factor_task_narrow_direct(const FactorJobDev& J, const float* const* segs,
                                                          int local, float* lds) {
  constexpr int NV = BK / (2 * NW);
  const int split = local;  // one tile
  const int64_t s0 = (int64_t)split * J.chunk;
  const int64_t s1 = min(J.nst, s0 + J.chunk);
  floatx16 acc[1];
#pragma unroll
  for (int v = 0; v < 16; ++v) acc[0][v] = 0.f;
  if (s1 > s0) {
    StageCursor c;
    c.init(J, s0);
    const float* base = seg_base(J, segs, c.seg);
    float cur[NV], nxt[NV];
    narrow_direct_load<NW>(J, base, c.k, seg_rows(J, c.seg), cur);
    for (int64_t s = s0; s < s1; ++s) {
      const int seg = c.seg;
      c.next(J.x.rows);
      if (s + 1 < s1) {
        if (c.seg != seg) base = seg_base(J, segs, c.seg);
        narrow_direct_load<NW>(J, base, c.k, seg_rows(J, c.seg), nxt);
      }
      if (s == J.rstage && s > s0) scale_acc(acc, J.rinv);  // (wave-uniform)
#pragma unroll
      for (int s2 = 0; s2 < NV; ++s2)
        acc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(cur[s2], cur[s2], acc[0], 0, 0, 0);
#pragma unroll
      for (int s2 = 0; s2 < NV; ++s2) cur[s2] = nxt[s2];
    }
    if (J.rstage >= 0 && s1 > J.rstage) scale_acc(acc, J.rw);
  }
  store_narrow<NW>(J, J.slab + (size_t)split * TILE * TILE, acc[0], lds);
}

// NSLOT ring slots (2: one stage in flight, 4 WGs/CU); one barrier per stage.
template <int GBK, int NSLOT>
__device__ __forceinline__ void factor_task_glds(const FactorJobDev& J, const float* const* segs,
                                                 int local, float* lds, int split_major) {
  static_assert(NSLOT >= 2, "ring must hold the computed stage and the next one");
  // split-major order: xcd_task hands every XCD a contiguous range of K-splits of
  // ALL tiles, so each XCD streams ~1/8 of the operand rows through its L2 once
  // (tile-major gave every XCD all K of its tiles' panels: ~8x the HBM fetch on
  // the multi-batch launches of a queued pass)
  const int ntiles = J.t * (J.t + 1) / 2;
  const int split = split_major ? local / ntiles : local % J.splits;
  const int tile = split_major ? local - split * ntiles : local / J.splits;
  int ti, tj;
  tri_decode(tile, ti, tj);
  const int64_t s0 = (int64_t)split * J.chunk;
  const int64_t s1 = min(J.nst, s0 + J.chunk);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // quadrant of this wave, rotated per dispatch round: the ~4 workgroups sharing a CU
  // put their idle quadrants (strictly-upper on diagonal tiles, tile padding) on
  // different SIMDs instead of all on the same one
  const int qw = (wave + (int)(blockIdx.x >> 8)) & 3;
  const int qi = qw >> 1, qj = qw & 1;
  const bool same = ti == tj;
  const bool active = !(same && qi < qj) && ti * TILE + qi * 32 < J.n && tj * TILE + qj * 32 < J.n;
  const bool narrow = J.n <= 32;  // one 32x32 quadrant: the 4 waves split K instead
  floatx16 acc;
#pragma unroll
  for (int v = 0; v < 16; ++v) acc[v] = 0.f;

  static_assert(GBK == BK, "a ring slot is one planner stage");
  if (s1 > s0) {
    // ring of NSLOT slots of GBK rows; NSLOT - 1 slots are in flight while a stage
    // computes.  Slots are issued and landed in stage order, each walked by its own
    // cursor across batch boundaries.
    constexpr int GSLOT = 2 * GBK * TILE;  // floats per ring slot (A and B panels)
    const int64_t rows = J.x.rows;
    GldsPanel<GBK> pa, pb;
    pa.init(J.x, ti * TILE, wave, lane, rows);
    pb.init(J.x, tj * TILE, wave, lane, rows);
    const int ns = (int)(s1 - s0);  // slots of this task
    const int per = (same ? 1 : 2) * GldsPanel<GBK>::NCH;  // LDS-DMA instructions per slot per thread
    StageCursor ic, fc;  // next slot to issue / to land
    ic.init(J, s0);
    fc = ic;
    const float* ibase = seg_base(J, segs, ic.seg);
    auto issue = [&](int sl) {
      float* slot = lds + (sl % NSLOT) * GSLOT;
      pa.issue(ibase, ic.k, slot, wave);
      if (!same) pb.issue(ibase, ic.k, slot + GBK * TILE, wave);
      const int seg = ic.seg;
      ic.next(rows);
      if (ic.seg != seg && sl + 1 < ns) ibase = seg_base(J, segs, ic.seg);
    };
#pragma unroll
    for (int p0 = 0; p0 < NSLOT - 1; ++p0)
      if (p0 < ns) issue(p0);
    const int h = lane >> 5, rr = lane & 31;
    for (int st = 0; st < ns; ++st) {
      // slot st landed; those issued after it may still fly
      const int issued = min(ns - 1, st + NSLOT - 2);
      vm_wait(per * (issued - st));
      float* slot = lds + (st % NSLOT) * GSLOT;
      pa.fixup(fc.k, slot);
      if (!same) pb.fixup(fc.k, slot + GBK * TILE);
      fc.next(rows);
      stage_barrier();  // stage st visible to all waves; everyone is done with stage st-1's slot
      if (st + NSLOT - 1 < ns) issue(st + NSLOT - 1);
      if (narrow) {
        const float* a = slot + h * TILE + rr;
#pragma unroll
        for (int s2 = 0; s2 < GBK / 8; ++s2) {
          const int ks = 2 * (wave * (GBK / 8) + s2);
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[ks * TILE], a[ks * TILE], acc, 0, 0, 0);
        }
      } else if (active) {
        const float* a = slot + h * TILE + qi * 32 + rr;
        const float* b = slot + (same ? 0 : GBK * TILE) + h * TILE + qj * 32 + rr;
        float av[GBK / 2], bv[GBK / 2];
#pragma unroll
        for (int s2 = 0; s2 < GBK / 2; ++s2) {
          av[s2] = a[2 * s2 * TILE];
          bv[s2] = b[2 * s2 * TILE];
        }
#pragma unroll
        for (int s2 = 0; s2 < GBK / 2; ++s2)
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[s2], bv[s2], acc, 0, 0, 0);
        // DS reads interleaved with the MFMAs (-1.2 us of 42 on the MLP update; a deeper
        // lookahead, the reads of MFMA pair t+2..4 issued with pair t, measured equal)
#pragma unroll
        for (int s2 = 0; s2 < GBK / 2; ++s2) {
          __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);  // 2 DS reads
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // 1 MFMA
        }
      }
    }
  }
  if (narrow) {  // (narrow => one tile, diagonal: A and B panels are the same)
    __syncthreads();
    store_narrow(J, J.slab + ((size_t)tile * J.sstride + split) * TILE * TILE, acc, lds);
    return;
  }
  if (!active) return;
  float* out = J.slab + ((size_t)tile * J.sstride + split) * TILE * TILE + qi * 32 * TILE + qj * 32;
  put_partial(J, acc, [&](int v) { return &out[acc_row(v, lane) * TILE + (lane & 31)]; });
}


// One launch per grouped update.  The row-major family (FAMILY = KFAC_ROWMAJOR)
// takes the LDS-DMA path when a job's operand allows it, else the register-staged
// row-major path; channel-major and im2col jobs get launches (and register budgets)
// of their own, instantiated per layout.  GLDS_ONLY: every job takes the LDS-DMA
// path (or the narrow direct-load path), and the ring is all the LDS (32 KB, not the
// register-staged path's 34 KB): 4 resident workgroups leave 32 KB of a CU's 160,
// room for a 32-tile inversion workgroup (29 KB) of an overlapped invert().
// Start delay per dispatch round (blockIdx / 256), in 512-cycle s_sleep(8) units: the
// workgroups that share a CU start ~1 us apart, so their load / barrier stalls
// interleave instead of coinciding (fp32 LDS-DMA SYRK: +2.5 %).  A design
// constant, not a timing build.
constexpr int STAGGER = 5;

template <int GBK, int NSLOT, bool GLDS_ONLY = false, int FAMILY = KFAC_ROWMAJOR>
__global__ __launch_bounds__(NTHREADS, 4) void kfac_factor_tiles_t(FactorArgs args) {
  constexpr int RING = FAMILY == KFAC_ROWMAJOR ? NSLOT * 2 * GBK * TILE : 0;
  constexpr int LDSF = GLDS_ONLY ? RING : ((4 * PANEL > RING) ? 4 * PANEL : RING);
  __shared__ __attribute__((aligned(16))) float lds[LDSF];
  // Workgroups of later dispatch rounds (blockIdx / 256: the ~4 sharing a CU) start a
  // fraction of a stage later, so their DMA waits and barriers interleave instead of
  // stalling all 16 waves of a CU together (measured +2.5% on the MLP update).
  for (int i = 0; i < STAGGER * (int)(blockIdx.x >> 8); ++i) __builtin_amdgcn_s_sleep(8);
  const int task = xcd_task(blockIdx.x, gridDim.x);
  int j = 0;
  while (j + 1 < args.njobs && task >= args.task_end[j]) ++j;
  const FactorJobDev& J = args.job[j];
  const int local = task - J.task_begin;
  if constexpr (FAMILY == KFAC_ROWMAJOR) {
    const float* const* segs = args.segs;
    if (J.glds)
      factor_task_glds<GBK, NSLOT>(J, segs, local, lds, args.split_major);
    else if constexpr (GLDS_ONLY)
      factor_task_narrow_direct(J, segs, local, lds);
    else
      factor_task<KFAC_ROWMAJOR>(J, segs, local, lds);
  } else {
    factor_task<FAMILY>(J, nullptr, local, lds);
  }
}

// production configuration: 32-row stages, 2-slot ring (one stage in flight)
#define kfac_factor_tiles kfac_factor_tiles_t<32, 2>
#define kfac_factor_tiles_glds kfac_factor_tiles_t<32, 2, true>
#define kfac_factor_tiles_channel kfac_factor_tiles_t<32, 2, false, KFAC_CHANNEL>
#define kfac_factor_tiles_patch kfac_factor_tiles_t<32, 2, false, KFAC_PATCH>

// ------------------------------------------------- bf16x3 split SYRK (row-major)
// fp32-accurate products on the bf16 matrix cores.  Every operand element is split
// EXACTLY into three bf16 parts, x = x1 + x2 + x3 (round-to-nearest splits: x1 holds
// the top 8 significant bits, x2 the next 8, x3 the last 8 of fp32's 24), and
//   x_a x_b = x1a x1b + (x1a x2b + x2a x1b) + (x1a x3b + x2a x2b + x3a x1b) + O(2^-24)
// -- six bf16 MFMA products per fp32 product, the dropped terms (x2 x3, x3 x2, x3 x3)
// below fp32's own rounding of the product, accumulated in fp32 by the MFMA.  On
// gfx950 v_mfma_f32_32x32x16_bf16 retires 16x the FLOP/cycle of the fp32 MFMA
// (v_mfma_f32_32x32x2_f32), so six of them are 2.67x the fp32 MFMA rate: the
// roofline of this kernel is 2.5 PF / 6 = 417 TF/s of fp32-equivalent work.
//
// kfac_factor_syrk3: one 128 x 128 macro tile (= 2 x 2 of the 64-tiles whose partial
// slabs the reduce sums) of one factor over one K-chunk per workgroup; the workgroup
// loads each 16-row substep of its panels once, splits it into the LDS image below and
// its 4 waves multiply from there (s3q_task).  Until round 5 a separate kfac_split3
// pass wrote the split images to HBM (6 B per operand element) and the SYRK read them
// back by LDS-DMA.
// LDS image of a substep: [part][column][2 chunks of 8 k] (32 B per column, k
// contiguous), read straight into MFMA operands (lane = column, 8 k per
// ds_read_b128); the chunk of a column is XOR-swizzled (s3_half), so the fragment
// reads and the split's writes are conflict-free and each read is a per-lane base plus
// an immediate.
// (A first version split in 8 producer waves beside 4 consumer waves per workgroup:
// producer-bound at 0.25 of the roofline)
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
constexpr int MT = 128;                          // macro tile edge
constexpr int S3_PART = 2 * MT * 32;             // bytes of one part of a substep slot (A and B)
constexpr int S3_REG = 3 * S3_PART + 64;         // one substep slot (+64: bank offset)

// byte offset of half-chunk hh (k 8hh .. 8hh+7 of a substep) of column c in a part.
// The half is swapped by bit 2 ^ bit 3 of the column: the fragment reads (ds_read_b128,
// lane groups {0-3, 12-15, 20-27} / {4-11, 16-19, 28-31}) and the split's writes
// (ds_write_b128, 8 consecutive columns) both hit distinct bank quads (bit 3 alone left
// the writes 2-way conflicted: 2.7 conflict cycles per LDS instruction, profiles/r06a_wide/)
__device__ __forceinline__ int s3_half(int c, int hh) { return c * 32 + ((hh ^ (((c >> 2) ^ (c >> 3)) & 1)) << 4); }

// (a, b) -> bf16 pair (a low), round to nearest even.  Inline asm: from a plain
// cast the compiler re-derives (pair << 16) as a second conversion of (a, 0)
__device__ __forceinline__ uint32_t bf16_pair(float a, float b) {
  uint32_t r;
  asm("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

// x - y as one v_sub_f32 (the compiler would pair the subtractions into
// v_pk_add_f32, which costs ~6x its issue slot beside MFMAs on gfx950; round 4, the
// residual pairs as explicit v_pk_add_f32: 169-171 vs 165-167 us per MLP launch)
__device__ __forceinline__ float sub_f32(float x, float y) {
  float r;
  asm("v_sub_f32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(y));
  return r;
}

// (a, b) -> their hi / mid / lo bf16 parts, packed as pairs (a low, b high).
// (x - part as one v_dot2c_f32_bf16, x + part * (-1) + 0 * other half, would save the
// expansion of each part: tried, but the instruction's result is not exact -- factor
// parity failed at 1.5e-4 relative -- so the residuals stay v_sub_f32.)
__device__ __forceinline__ void split3(float a, float b, uint32_t& h, uint32_t& m, uint32_t& l) {
  h = bf16_pair(a, b);
  const float ra = sub_f32(a, __uint_as_float(h << 16)), rb = sub_f32(b, __uint_as_float(h & 0xffff0000u));
  m = bf16_pair(ra, rb);
  const float sa = sub_f32(ra, __uint_as_float(m << 16)), sb = sub_f32(rb, __uint_as_float(m & 0xffff0000u));
  l = bf16_pair(sa, sb);
}

// A wave's MFMAs on one 16-row k-substep (the slot at `reg`): blocks (bi, bj) of its
// 64 x 64 quadrant with act[bi][bj], six products per block.  oa / ob: this lane's A / B
// fragment offsets (part 0, block 0); everything else is an immediate.  The 12
// fragments go out first, then the MFMAs.
__device__ __forceinline__ void s3_consume_sub(const char* reg, int oa, int ob, const bool (&act)[2][2],
                                               floatx16 (&acc)[2][2]) {
  auto frag = [&](int off) { return *reinterpret_cast<const bf16x8*>(reg + off); };
  auto six = [&](int bi, int bj, const bf16x8* A, const bf16x8* B) {
    if (!act[bi][bj]) return;
    acc[bi][bj] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[2], B[0], acc[bi][bj], 0, 0, 0);
    acc[bi][bj] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[1], B[1], acc[bi][bj], 0, 0, 0);
    acc[bi][bj] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[0], B[2], acc[bi][bj], 0, 0, 0);
    acc[bi][bj] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[1], B[0], acc[bi][bj], 0, 0, 0);
    acc[bi][bj] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[0], B[1], acc[bi][bj], 0, 0, 0);
    acc[bi][bj] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[0], B[0], acc[bi][bj], 0, 0, 0);
  };
  bf16x8 a0[3], a1[3], b0[3], b1[3];
#pragma unroll
  for (int p = 0; p < 3; ++p) {
    a0[p] = frag(oa + p * S3_PART);
    b0[p] = frag(ob + p * S3_PART);
    b1[p] = frag(ob + p * S3_PART + 32 * 32);
    a1[p] = frag(oa + p * S3_PART + 32 * 32);
  }
  six(0, 0, a0, b0);
  six(0, 1, a0, b1);
  six(1, 0, a1, b0);
  six(1, 1, a1, b1);
}

// Macro tile of a unit index, in blocks of 4 tile rows x 8 tile columns of the lower
// triangle: the ~32 tasks an XCD runs at once (xcd_task hands it a contiguous range)
// then read 4 A panels and 8 B panels, not 1 and 32, so a stage's rows are fetched
// into its L2 once per panel block instead of once per task (wide factors: 4096
// columns = 32 panels of 128 each far larger than the 4 MB L2).
__device__ __forceinline__ void s3_decode(int unit, int T3, int& I, int& J) {
  int base = 0;
  I = J = 0;
  for (int i0 = 0; i0 < T3; i0 += 4) {
    const int i1 = min(T3, i0 + 4);
    for (int j0 = 0; j0 < i1; j0 += 8) {
      int cnt = 0;
      for (int i = i0; i < i1; ++i) cnt += max(0, min(j0 + 8, i + 1) - j0);
      if (unit < base + cnt) {
        int r = unit - base;
        for (int i = i0; i < i1; ++i) {
          const int w = max(0, min(j0 + 8, i + 1) - j0);
          if (r < w) {
            I = i;
            J = j0 + r;
            return;
          }
          r -= w;
        }
      }
      base += cnt;
    }
  }
}

// ------------------------------------- bf16x3 SYRK, split once per workgroup
// (round 5; replaces the separate split pass).  One 128 x 128 macro
// tile of one factor over one K-chunk per workgroup of 4 waves, 2 workgroups per CU.
// Per 16-row substep, thread t loads column t of the [A panel | B panel] (256 columns)
// -- 16 rows, two 8-row halves, buffer loads whose record limit zero-fills rows past
// the batch and columns past the operand -- splits it into its three bf16 parts and
// writes them as the substep's LDS image (the layout above: [part][column][2 halves],
// half swizzled by bit 3 of the column).  Two slots: while the waves' MFMAs consume
// substep h from one, the split of substep h + 1 goes into the other, interleaved with
// those MFMAs (sched_group_barrier), and the loads of substep h + 2 are in flight.
// One barrier per substep.  Each wave computes its 64 x 64 quadrant (w >> 1, w & 1)
// as 2 x 2 blocks, six products per block: 24 MFMAs per substep against 2 columns x
// 16 values split per thread (3.7 VALU per MFMA; tools/microbench/cutq_mb.hip: 0.448
// of 417 TF/s on a 4096-column operand).
constexpr int KFAC_S3D_WGS = 2;  // resident workgroups per CU the planner counts on
constexpr int S3D_WGS = KFAC_S3D_WGS;
constexpr int S3D_LDS = 2 * S3_REG;

template <bool FILL>
__device__ __forceinline__ void s3q_task(const FactorJobDev& J, const float* const* segs, int local,
                                         char* lds) {
  const int T3 = (J.n + MT - 1) / MT, units = T3 * (T3 + 1) / 2;
  const int split = local / units, unit = local - split * units;
  int I, Jc;
  s3_decode(unit, T3, I, Jc);
  const int64_t s0 = (int64_t)split * J.chunk;
  const int64_t s1 = min(J.nst, s0 + J.chunk);
  const int nh = 2 * (int)(s1 - s0);  // 16-row substeps (even)
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 1, wc = wave & 1;
  bool act[2][2];
#pragma unroll
  for (int bi = 0; bi < 2; ++bi)
#pragma unroll
    for (int bj = 0; bj < 2; ++bj) {
      const int r0 = I * MT + wr * 64 + bi * 32, c0 = Jc * MT + wc * 64 + bj * 32;
      act[bi][bj] = r0 < J.n && c0 < J.n && r0 >= c0;
    }
  floatx16 acc[2][2];
#pragma unroll
  for (int bi = 0; bi < 2; ++bi)
#pragma unroll
    for (int bj = 0; bj < 2; ++bj)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[bi][bj][v] = 0.f;
  // this thread's column of the [A | B] panels
  const int ld4 = (int)J.x.ld * 4;
  const int rows = (int)J.x.rows;
  const int rec = rows * ld4;  // a batch's bytes (planner: < 2^31)
  const int gc = tid < MT ? I * MT + tid : Jc * MT + (tid - MT);
  const int voff = gc < J.x.cols ? gc * 4 : rec;  // past the operand: the zero tail
  const bool ones = gc == J.x.ones;
  const int wo = s3_half(tid, 0), wo1 = s3_half(tid, 1);
  // substep cursor: batch `seg` (base `b`), first row `k` of the substep within it
  const int sub_per_seg = 2 * J.sps;
  int seg = (int)(s0 / J.sps);
  int k = (int)((s0 - (int64_t)seg * J.sps) * BK);
  const int lastseg = J.nseg - 1;
  const float* b = seg_base(J, segs, seg);
  const float* nb = seg_base(J, segs, min(seg + 1, lastseg));  // the next batch's base
  int left = nh - 1;  // substeps after the cursor's within the task (it stops at the last)
  int ksub = k / 16;  // substep index within the batch
  // branch-free (scalar selects): a branch here splits the loop body and the compiler
  // then copies the load register sets at the join
  auto advance = [&]() {
    const int more = left > 0;
    left -= more;
    ksub += more;
    k += 16 * more;
    const bool wrap = ksub == sub_per_seg;
    ksub = wrap ? 0 : ksub;
    k = wrap ? 0 : k;
    seg += wrap;
    b = wrap ? nb : b;
    nb = seg_base(J, segs, min(seg + 1, lastseg));
  };
  struct Sub {
    int seg, k;
  };
  auto load = [&](float (&L)[2][8]) {
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(b), 0, rec, 0x00020000);
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int r = 0; r < 8; ++r)
        L[u][r] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, voff, (k + 8 * u + r) * ld4, 0));
  };
  auto put1 = [&](float (&x)[8], int u, const Sub& sb, char* slot) {
    if constexpr (FILL) {  // the ones column: 1 on the batch's rows, 0 past them
      const int nvalid = (int)seg_rows(J, sb.seg) - sb.k - 8 * u;
#pragma unroll
      for (int r = 0; r < 8; ++r) x[r] = ones ? (r < nvalid ? 1.f : 0.f) : x[r];
    }
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    u32x4 hp, mp, lp;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      uint32_t a2, b2, c2;
      split3(x[2 * i], x[2 * i + 1], a2, b2, c2);
      hp[i] = a2;
      mp[i] = b2;
      lp[i] = c2;
    }
    const int o = u ? wo1 : wo;
    *reinterpret_cast<u32x4*>(slot + o) = hp;
    *reinterpret_cast<u32x4*>(slot + S3_PART + o) = mp;
    *reinterpret_cast<u32x4*>(slot + 2 * S3_PART + o) = lp;
  };
  const int lo = s3_half(lane & 31, lane >> 5);
  const int oa = wr * 64 * 32 + lo, ob = (MT + wc * 64) * 32 + lo;
  auto frag = [&](const char* slot, int off) { return *reinterpret_cast<const bf16x8*>(slot + off); };
  float L0[2][8], L1[2][8];
  Sub sub0{seg, k}, sub1;
  load(L0);
  advance();
  sub1 = Sub{seg, k};
  load(L1);
  advance();
  asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // L0 landed
  put1(L0[0], 0, sub0, lds);
  put1(L0[1], 1, sub0, lds);
  __syncthreads();
  // substep hs: MFMAs from slot hs & 1; Lsplit (substep hs + 1) split into the other
  // slot during them; Lload refilled with substep hs + 2
  auto body = [&](int hs, float (&Lsplit)[2][8], const Sub& ssplit, float (&Lload)[2][8]) {
    const char* cur = lds + (hs & 1) * S3_REG;
    char* nxt = lds + ((hs + 1) & 1) * S3_REG;
    bf16x8 A[2][3], B[2][3];
#pragma unroll
    for (int p = 0; p < 3; ++p) A[0][p] = frag(cur, oa + p * S3_PART);
    load(Lload);  // (past the task's rows: the last substep again, never used)
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // Lsplit has landed
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int bi = 0; bi < 2; ++bi) {
      if (bi == 0)
#pragma unroll
        for (int p = 0; p < 3; ++p) A[1][p] = frag(cur, oa + p * S3_PART + 32 * 32);
#pragma unroll
      for (int bj = 0; bj < 2; ++bj) {
        if (bi == 0)
#pragma unroll
          for (int p = 0; p < 3; ++p) B[bj][p] = frag(cur, ob + p * S3_PART + bj * 32 * 32);
        const bf16x8* Aa = A[bi];
        acc[bi][bj] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(Aa[2], B[bj][0], acc[bi][bj], 0, 0, 0);
        acc[bi][bj] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(Aa[1], B[bj][1], acc[bi][bj], 0, 0, 0);
        acc[bi][bj] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(Aa[0], B[bj][2], acc[bi][bj], 0, 0, 0);
        acc[bi][bj] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(Aa[1], B[bj][0], acc[bi][bj], 0, 0, 0);
        acc[bi][bj] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(Aa[0], B[bj][1], acc[bi][bj], 0, 0, 0);
        acc[bi][bj] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(Aa[0], B[bj][0], acc[bi][bj], 0, 0, 0);
      }
      // (unconditional: past the last substep it fills the free slot -- a branch here
      // made the compiler copy the 64 accumulators every trip)
      put1(Lsplit[bi], bi, ssplit, nxt);
      // pattern: the fragment reads first, then per MFMA ~4 VALU of the split, a DS
      // write every 4 MFMAs
      if (bi == 0) __builtin_amdgcn_sched_group_barrier(0x100, 6, 0);
#pragma unroll
      for (int i = 0; i < 12; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        if (bi == 0 && i == 5) __builtin_amdgcn_sched_group_barrier(0x100, 6, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);
        if (i % 4 == 3) __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    __syncthreads();
  };
  for (int hs = 0; hs < nh; hs += 2) {
    const Sub s2{seg, k};
    body(hs, L1, sub1, L0);  // L0 <- substep hs + 2
    advance();
    sub0 = s2;
    const Sub s3{seg, k};
    body(hs + 1, L0, sub0, L1);  // L1 <- substep hs + 3
    advance();
    sub1 = s3;
  }
  const int ti = 2 * I + wr, tj = 2 * Jc + wc;
  float* o = J.slab + ((size_t)(ti * (ti + 1) / 2 + tj) * J.sstride + split) * TILE * TILE;
#pragma unroll
  for (int bi = 0; bi < 2; ++bi)
#pragma unroll
    for (int bj = 0; bj < 2; ++bj)
      if (act[bi][bj])
        put_partial(J, acc[bi][bj],
                    [&](int v) { return &o[(bi * 32 + acc_row(v, lane)) * TILE + bj * 32 + (lane & 31)]; });
}

__global__ __launch_bounds__(NTHREADS, S3D_WGS) void kfac_factor_syrk3(FactorArgs args) {
  extern __shared__ __attribute__((aligned(16))) char s3lds[];
  const int task = xcd_task(blockIdx.x, gridDim.x);
  int j = 0;
  while (j + 1 < args.njobs && task >= args.task_end[j]) ++j;
  const FactorJobDev& J = args.job[j];
  const int local = task - J.task_begin;
  if (J.n <= 32) {
    factor_task_narrow_direct(J, args.segs, local, reinterpret_cast<float*>(s3lds));
    return;
  }
  // the macro tile whose panels hold the ones column splits with the fill
  const int T3 = (J.n + MT - 1) / MT, units = T3 * (T3 + 1) / 2;
  int I, Jc;
  s3_decode(local % units, T3, I, Jc);
  const int o = J.x.ones;
  const bool fill = o >= 0 && (o / MT == I || o / MT == Jc);
  if (fill)
    s3q_task<true>(J, args.segs, local, s3lds);
  else
    s3q_task<false>(J, args.segs, local, s3lds);
}

// ------------------------------- fp32 operands, bf16x3 products split in registers
// kfac_factor_tiles_x3: TWO waves per 64 x 64 tile, each computing the WHOLE tile over
// its own 16-row half of every 32-row stage.  A lane loads its MFMA fragment -- 8
// consecutive k of one column -- straight from global memory into registers (no LDS),
// splits it (split3: the exact three-part split of the bf16x3 kernels above) and the
// wave runs six v_mfma_f32_32x32x16_bf16 per 32 x 32 block: 24 MFMAs of 32 cycles per
// wave and 16-row half, against the fp32 kernel's 4 waves x 8 fp32 MFMAs of 64 cycles
// for the same work, with no split pass and no padded images (the n <= 1024 factors,
// where kfac_split3's HBM round trip costs as much as the products).  The two waves'
// partial tiles are summed through LDS in a fixed order at the end.
// Measured on the MNIST MLP group (profiles/r03_x3/ab/probe_summary.txt): direct loads
// beat LDS-DMA rings (shared, one barrier per stage, or one per wave without a
// barrier: 179 vs 196-204 us per 32,768-row launch), the compiled split beats a
// hand-ordered asm one, and 128 x 128 macro tiles with the split made once per macro
// tile into the syrk3 LDS image (x3m) lost (224 us).  The kernel is issue-bound: two
// waves per SIMD keep its issue port ~90 % busy with 7.3 split VALU per MFMA.
constexpr int X3_THREADS = 128;

// kfac_factor_tiles_x3's work units of a factor of n over T = ceil(n / 64) tiles per
// edge: the lower-triangle tiles, or with a thin last tile row (T >= 2 and at most 32
// rows in it) the T-1 pairs (i, i) + (T-1, i), the other strictly lower tiles of rows
// < T-1 and the corner (see X3_PAIR)
static inline bool x3_thin(int n, int T) { return T >= 2 && n - TILE * (T - 1) <= 32; }
// a thin-row x3 job with f full-tile K-splits gets S = f + f / k slabs per tile, the last
// f / k of them written by extra K-splits of its pair units only; k = 5 (MNIST MLP, same
// box, 200 steps: 3 / 5 / 10 / none 145.7 / 145.6 / 150.0 / 153.1 us per launch,
// DESIGN.md 3.1c)
constexpr int X3_PAIR_XS = 5;
static inline int x3_pair_xs() { return X3_PAIR_XS; }
// S / (k + 1) recovers f / k from S = f + f / k (f = k a + b, b <= k - 1)
static inline int64_t x3_xsplits(int64_t S) { return x3_pair_xs() ? S / (x3_pair_xs() + 1) : 0; }
__host__ __device__ inline int x3_units_of(int T, bool pair) { return T * (T + 1) / 2 - (pair ? T - 1 : 0); }
static inline int x3_units(int n, int T) { return x3_units_of(T, x3_thin(n, T)); }
constexpr int X3_NW = X3_THREADS / 64;

struct X3Frag {
  bf16x8 p[3];  // hi, mid, lo
};

__device__ __forceinline__ void x3_six(floatx16& acc, const X3Frag& A, const X3Frag& B) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A.p[2], B.p[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A.p[1], B.p[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A.p[0], B.p[2], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A.p[1], B.p[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A.p[0], B.p[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A.p[0], B.p[0], acc, 0, 0, 0);
}

// The same for a diagonal block (A = B): the cross products come in transposed pairs
// (lo hi^T and hi lo^T, mid hi^T and hi mid^T), so four MFMAs -- hh + mm into acc,
// (lo + mid) hi^T into acc2 -- and the caller adds acc2 + acc2^T once at the end.
__device__ __forceinline__ void x3_four(floatx16& acc, floatx16& acc2, const X3Frag& A) {
  acc2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A.p[2], A.p[0], acc2, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A.p[1], A.p[1], acc, 0, 0, 0);
  acc2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A.p[1], A.p[0], acc2, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A.p[0], A.p[0], acc, 0, 0, 0);
}

// Operands straight from global memory into registers, no LDS: a lane's fragment is
// rows kw .. kw+7 of one column, eight buffer loads that differ only in their SGPR
// offset (r * ld * 4 bytes), so the addressing costs no VALU; the buffer's record
// limit (the batch's bytes) zero-fills rows past the batch.  The next stage's
// fragments are loaded while the current ones are split and multiplied.
struct X3Col {
  int voff;  // byte offset of (row 16 wave + 8 h, column) from the batch base
  bool fill; // a column past the operand's data (fill value instead)
  float fv;  // its fill value (the ones column: 1)
};

__device__ __forceinline__ void x3_load8(float (&x)[8], __amdgpu_buffer_rsrc_t rs, const X3Col& c,
                                         int sbase, int sstep) {
#pragma unroll
  for (int r = 0; r < 8; ++r)
    x[r] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, c.voff, sbase + r * sstep, 0));
}

// (a hand-ordered asm split with no cvt -> use pads measured slower, 195 vs 181 us
// per 32,768-row MLP launch: the compiler interleaves the split with the MFMAs)
__device__ __forceinline__ X3Frag x3_split8(const float (&x)[8]) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  u32x4 h, m, l;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    uint32_t a, b, c;
    split3(x[2 * i], x[2 * i + 1], a, b, c);
    h[i] = a;
    m[i] = b;
    l[i] = c;
  }
  X3Frag f;
  f.p[0] = __builtin_bit_cast(bf16x8, h);
  f.p[1] = __builtin_bit_cast(bf16x8, m);
  f.p[2] = __builtin_bit_cast(bf16x8, l);
  return f;
}

// The stage loop (round 4): software-pipelined segments in ONE straight-line block.
// The fragments of the stage's first block -- A0 (and B0) -- are split during the
// previous stage; every segment is the six MFMAs of one block interleaved
// (sched_group_barrier) with the split of a fragment a later block needs, and that
// fragment's registers are reloaded as soon as its split has read them:
//   full tile (mask 15):  (0,0) | split A1    (1,0) | split B1    (0,1) | split A0'
//                         (1,1) | split B0'
// so each load goes out one whole stage before its split (x1, x3 hold the next stage,
// x0, x2 the one after), at most five fragments are live and no register set is copied
// (2 waves per SIMD at <= 200 VGPRs leave an inversion wave room beside them).  Round 3's
// loop split all four fragments at the top of the stage, copied a 32-register prefetch
// set into the working set every stage, branched per stage (last stage, batch change,
// fill columns with 64-bit compares), and the compiler sank every load to the end of
// the body and waited vmcnt(0) at the loop head: ~100 extra VALU and the whole L2
// latency per stage.  Now every load is unconditional: past the task's range the
// cursor stops (the last stage reloads itself), a batch change is a scalar select (the
// next batch's base fetched a stage ahead), columns past the operand load from past
// the buffer's record limit (0), and the ones column (FILL: only the tasks whose
// fragments hold it) is a select of 1 / 0 by row validity.
// Microbench: tools/microbench/x3w_mb.hip; DESIGN.md §3.1c.
struct X3Cursor {  // a stage to load: batch `seg` (base `b`), first row `k`
  const float* b;
  int seg, k;
};

template <int NV>
__device__ __forceinline__ void x3_pattern() {  // 6 MFMAs, NV VALU each, the reloads early
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);       // MFMA
    if (NV > 0) __builtin_amdgcn_sched_group_barrier(0x002, NV, 0);  // VALU
    // (all 8 reloads after the first MFMA: 170 vs 159-166 us, profiles/r04v/)
    if (i < 4) __builtin_amdgcn_sched_group_barrier(0x020, 2, 0);  // VMEM read
  }
}

// X3_PAIR: a factor whose last tile row is thin (n - 64 (T-1) <= 32: one block row,
// the MNIST MLP's 785 and 129) pairs diagonal tile (i, i) with edge tile (T-1, i) in ONE
// task: fragments A0, A1 (panel i) and C0 (panel T-1, block 0), five blocks
//   D00 = A0 A0, D10 = A1 A0, D11 = A1 A1 (tile (i, i)), E00 = C0 A0, E01 = C0 A1
// -- 30 MFMAs on 3 fragments per 16 rows, where the diagonal task alone did 18 on 2
// and the edge task 12 on 3 (both ran ahead of the full tiles, widening each XCD's
// L2 working set), and T-1 fewer tasks per K-split.  acc[0][0] D00, acc[1][0] D10,
// acc[1][1] D11, acc[0][1] E00, acc4 E01; called with ti = i, tj = T-1.
constexpr int X3_PAIR = 16;

template <int MASK, bool FILL>
__device__ __forceinline__ void x3_loop(const FactorJobDev& J, const float* const* segs, int ti, int tj,
                                        int64_t s0, int64_t s1, floatx16 (&acc)[2][2], floatx16& acc4) {
  constexpr bool PAIR = MASK == X3_PAIR;
  constexpr bool A00 = MASK & 1, A01 = MASK & 2, A10 = MASK & 4, A11 = MASK & 8;
  constexpr bool ROW1 = A10 || A11 || PAIR, COL1 = A01 || A11;
  // masks 13 and 1 occur on diagonal tiles only (an off-diagonal tile with block
  // (1, 1), or with any block, has (0, 1)): B fragments = A fragments
  constexpr bool SAME = MASK == 13 || MASK == 1;
  static_assert(A00 || PAIR, "block (0, 0) always has work");
  // fragments: 0 A block 0, 1 A block 1, 2 B block 0, 3 B block 1 (PAIR: 2 = C0)
  constexpr bool USE[4] = {true, ROW1, !SAME, !SAME && COL1};
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int ld4 = (int)J.x.ld * 4;
  const int rows = (int)J.x.rows;
  const int rec = rows * ld4;                  // a batch's bytes (planner: < 2^31)
  // (the ragged last batch's: its rows past x.last_rows read as zeros)
  const int rec_last = rec - J.rdelta * ld4;
  const int lr = 16 * wave + 8 * (lane >> 5);  // lane's first row within a stage
  int voff[4];
  bool onesl[4];
#pragma unroll
  for (int f = 0; f < 4; ++f) {
    const int c = (f < 2 ? ti : tj) * TILE + (f & 1) * 32 + (lane & 31);
    voff[f] = c < J.x.cols ? lr * ld4 + c * 4 : rec;  // past the operand: the zero tail
    onesl[f] = c == J.x.ones;
  }
  const int ns = (int)(s1 - s0);
  const int lastseg = J.nseg - 1;
  // stage cursors: c1 = the next stage to load for fragments 1 / 3, c2 = the one after
  // (fragments 0 / 2); nb = the base of the batch after c2's
  X3Cursor c2;
  c2.seg = (int)(s0 / J.sps);
  c2.k = (int)((s0 - (int64_t)c2.seg * J.sps) * BK);
  c2.b = seg_base(J, segs, c2.seg);
  const float* nb = seg_base(J, segs, min(c2.seg + 1, lastseg));
  int left = ns - 1;  // stages after c2's within the task (the cursor stops at the last)
  auto advance = [&](X3Cursor& c) {
    const bool more = left > 0;
    const bool wrap = more && c.k + BK >= rows;
    c.k = more ? (wrap ? 0 : c.k + BK) : c.k;
    c.seg += wrap;
    c.b = wrap ? nb : c.b;
    nb = seg_base(J, segs, min(c.seg + 1, lastseg));
    left -= more;
  };
  auto rsrc = [&](const float* b, int seg) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(b), 0, seg == lastseg ? rec_last : rec,
                                             0x00020000);
  };
  auto ld8 = [&](int f, const X3Cursor& c, float (&x)[8]) {
    x3_load8(x, rsrc(c.b, c.seg), X3Col{voff[f], false, 0.f}, c.k * ld4, ld4);
  };
  float x[4][8];
  // prologue: stage s0 into every fragment, the first block's fragments split, their
  // registers reloaded with stage s0 + 1
  const int k0 = c2.k, seg0 = c2.seg;
#pragma unroll
  for (int f = 0; f < 4; ++f)
    if (USE[f]) ld8(f, c2, x[f]);
  advance(c2);
  X3Cursor c1 = c2;  // (fragments 1 / 3 load stage s0 + 1 in the first stage)
  int kc = k0, kcs = seg0;  // first row and batch of the stage being multiplied
  auto fix = [&](int f, int kstage, int kseg) {  // the ones column: 1 on the batch's rows, 0 past them
    if constexpr (FILL) {
      const int nvalid = (int)seg_rows(J, kseg) - kstage;
#pragma unroll
      for (int r = 0; r < 8; ++r) x[f][r] = onesl[f] ? (lr + r < nvalid ? 1.f : 0.f) : x[f][r];
    }
  };
  // split fragment f (of the stage starting at row kstage of batch kseg) and reload its
  // registers
  auto take = [&](int f, int kstage, int kseg, const X3Cursor& c) {
    fix(f, kstage, kseg);
    const X3Frag fr = x3_split8(x[f]);
    ld8(f, c, x[f]);
    return fr;
  };
  X3Frag pa = take(0, k0, seg0, c2);
  X3Frag pb = SAME ? pa : take(2, k0, seg0, c2);
  // the prologue's loads complete here (once per task): the loop header then starts
  // from a precise wait state, and the compiler keeps the counted vmcnt at the top of
  // each stage (with the prologue's loads still in flight it merged them into a
  // vmcnt(0) there, exposing a whole stage of load latency)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  // (6 / 11 VALU slots per MFMA measured equal within the box's +-4 us, profiles/r04v/)
  constexpr int NV = FILL ? 52 / 6 + 1 : 44 / 6 + 1;
  // one stage: P = (A0, B0) of this stage in, (A0', B0') of the next stage out
  auto stage = [&](const X3Frag& A0, const X3Frag& B0, X3Frag& A0n, X3Frag& B0n) {
    const int kn = c2.k, kns = c2.seg;  // first row / batch of the next stage (in x0 / x2 now)
    // the cursors: x1 / x3 reload the next stage, x0 / x2 the one after
    c1 = c2;
    advance(c2);
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (PAIR) {  // B0 = C0
      const X3Frag A1 = take(1, kc, kcs, c1);
      x3_six(acc[0][0], A0, A0);
      x3_pattern<NV>();
      __builtin_amdgcn_sched_barrier(0);
      A0n = take(0, kn, kns, c2);
      x3_six(acc[0][1], B0, A0);
      x3_pattern<NV>();
      __builtin_amdgcn_sched_barrier(0);
      B0n = take(2, kn, kns, c2);
      x3_six(acc[1][0], A1, A0);
      x3_pattern<NV>();
      __builtin_amdgcn_sched_barrier(0);
      x3_six(acc[1][1], A1, A1);
      x3_pattern<0>();
      __builtin_amdgcn_sched_barrier(0);
      x3_six(acc4, B0, A1);
      x3_pattern<0>();
    } else if constexpr (MASK == 15) {
      const X3Frag A1 = take(1, kc, kcs, c1);
      x3_six(acc[0][0], A0, B0);
      x3_pattern<NV>();
      __builtin_amdgcn_sched_barrier(0);
      const X3Frag B1 = take(3, kc, kcs, c1);
      x3_six(acc[1][0], A1, B0);
      x3_pattern<NV>();
      __builtin_amdgcn_sched_barrier(0);
      A0n = take(0, kn, kns, c2);
      x3_six(acc[0][1], A0, B1);
      x3_pattern<NV>();
      __builtin_amdgcn_sched_barrier(0);
      B0n = take(2, kn, kns, c2);
      x3_six(acc[1][1], A1, B1);
      x3_pattern<NV>();
    } else if constexpr (MASK == 13) {  // diagonal: (0,0) (1,0) (1,1), B = A
      const X3Frag A1 = take(1, kc, kcs, c1);
      x3_six(acc[0][0], A0, A0);
      x3_pattern<NV>();
      __builtin_amdgcn_sched_barrier(0);
      x3_six(acc[1][0], A1, A0);
      A0n = take(0, kn, kns, c2);
      x3_pattern<NV>();
      __builtin_amdgcn_sched_barrier(0);
      x3_six(acc[1][1], A1, A1);
      x3_pattern<0>();
      B0n = A0n;
    } else if constexpr (MASK == 5) {  // (0,0) (1,0)
      const X3Frag A1 = take(1, kc, kcs, c1);
      x3_six(acc[0][0], A0, B0);
      x3_pattern<NV>();
      __builtin_amdgcn_sched_barrier(0);
      A0n = take(0, kn, kns, c2);
      B0n = take(2, kn, kns, c2);
      x3_six(acc[1][0], A1, B0);
      x3_pattern<2 * NV>();
    } else if constexpr (MASK == 3) {  // (0,0) (0,1): the last tile row of a factor
      const X3Frag B1 = take(3, kc, kcs, c1);
      x3_six(acc[0][0], A0, B0);
      x3_pattern<NV>();
      __builtin_amdgcn_sched_barrier(0);
      A0n = take(0, kn, kns, c2);
      B0n = take(2, kn, kns, c2);
      x3_six(acc[0][1], A0, B1);
      x3_pattern<2 * NV>();
    } else {  // 1: the last diagonal tile, (0,0) only, B = A
      A0n = take(0, kn, kns, c2);
      x3_six(acc[0][0], A0, A0);
      x3_pattern<NV>();
      B0n = A0n;
    }
    kc = kn;
    kcs = kns;
  };
  // the ragged last batch: sums so far scaled by 1 / rw where the task crosses into it,
  // everything by rw at the end when it reaches it (FactorJobDev::rstage)
  const int64_t rst = J.rstage;
  const int bst = (rst > s0 && rst < s1) ? (int)(rst - s0) : -1;
  for (int st = 0; st < ns; ++st) {
    if (st == bst) {
      scale_acc(acc[0], J.rinv);
      scale_acc(acc[1], J.rinv);
      if constexpr (PAIR) {
        floatx16 a4[1] = {acc4};
        scale_acc(a4, J.rinv);
        acc4 = a4[0];
      }
    }
    X3Frag qa, qb;
    stage(pa, pb, qa, qb);
    pa = qa;
    pb = qb;
  }
  if (rst >= 0 && s1 > rst) {
    scale_acc(acc[0], J.rw);
    scale_acc(acc[1], J.rw);
    if constexpr (PAIR) {
      floatx16 a4[1] = {acc4};
      scale_acc(a4, J.rw);
      acc4 = a4[0];
    }
  }
}

template <int GBK, int NSLOT>
__device__ __forceinline__ void factor_task_x3(const FactorJobDev& J, const float* const* segs, int local,
                                               float* lds, int split_major) {
  static_assert(GBK == 16 * X3_NW, "one 16-row half stage per wave");
  const int T = J.t;
  const bool thin = J.x3pair != 0;
  const int units = x3_units_of(T, thin);
  const int sf = J.splits - J.xsplits;  // the full K-splits (every unit)
  int split, unit;
  if (local >= units * sf) {  // the pair units' extra K-splits (x3_xsplits)
    const int e = local - units * sf;
    split = sf + e / (T - 1);
    unit = e - (split - sf) * (T - 1);
  } else {
    split = split_major ? local / units : local % sf;
    unit = split_major ? local - split * units : local / sf;
  }
  int ti, tj;
  bool pair = false;
  if (!thin) {
    tri_decode(unit, ti, tj);
  } else if (unit < T - 1) {  // pairs first: diagonal (i, i) with edge (T-1, i)
    pair = true;
    ti = unit;
    tj = T - 1;
  } else if (unit < T - 1 + (T - 1) * (T - 2) / 2) {  // strictly lower tiles of rows < T-1
    tri_decode(unit - (T - 1), ti, tj);
    ++ti;  // (row i of the strict lower triangle has i tiles: tri index of (i-1, j))
  } else {  // the corner (T-1, T-1)
    ti = tj = T - 1;
  }
  const int tile = ti * (ti + 1) / 2 + (pair ? ti : tj);  // (a pair's: its diagonal tile)
  // a pair unit's K-chunk: nst over all `splits` slabs; the others' over the full splits
  const int64_t chunk = pair && J.xsplits ? (J.nst + J.splits - 1) / J.splits : J.chunk;
  const int64_t s0 = (int64_t)split * chunk;
  const int64_t s1 = min(J.nst, s0 + chunk);
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const bool same = ti == tj;
  bool act[2][2];
  int mask = 0;
#pragma unroll
  for (int bi = 0; bi < 2; ++bi)
#pragma unroll
    for (int bj = 0; bj < 2; ++bj) {
      act[bi][bj] = !(same && bi < bj) && ti * TILE + bi * 32 < J.n && tj * TILE + bj * 32 < J.n;
      mask |= act[bi][bj] << (2 * bi + bj);
    }
  if (pair) mask = X3_PAIR;
  floatx16 acc[2][2], acc4;
#pragma unroll
  for (int bi = 0; bi < 2; ++bi)
#pragma unroll
    for (int bj = 0; bj < 2; ++bj)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[bi][bj][v] = 0.f;
#pragma unroll
  for (int v = 0; v < 16; ++v) acc4[v] = 0.f;
  if (s1 > s0) {
    // FILL: one of the task's fragments holds the ones column (the last tile row /
    // column of an A factor with a bias)
    const bool fill = J.x.ones >= 0 && ((J.x.ones >> 6) == ti || (J.x.ones >> 6) == tj);
#define X3_CASE(M)                                                   \
  case M:                                                            \
    if (fill) x3_loop<M, true>(J, segs, ti, tj, s0, s1, acc, acc4);  \
    else x3_loop<M, false>(J, segs, ti, tj, s0, s1, acc, acc4);      \
    break;
    switch (mask) {  // (block (0, 0) always has work)
      X3_CASE(X3_PAIR)
      X3_CASE(15)
      X3_CASE(13)  // diagonal
      X3_CASE(5)
      X3_CASE(3)
      X3_CASE(1)
      default: break;  // (not reached)
    }
#undef X3_CASE
  }
  if (pair) {
    // wave 0 keeps D00, E00, E01 and wave 1 D10, D11; each hands the other's through
    // LDS slots [D00, D10, D11, E00, E01][16 values][64 lanes]; sums are w0 + w1
    __syncthreads();
    float* xo = lds;
    auto put = [&](int sl, const floatx16& a) {
#pragma unroll
      for (int v = 0; v < 16; ++v) xo[(sl * 16 + v) * 64 + lane] = a[v];
    };
    auto add = [&](int sl, floatx16& a) {
#pragma unroll
      for (int v = 0; v < 16; ++v) a[v] += xo[(sl * 16 + v) * 64 + lane];
    };
    float* outD = J.slab + ((size_t)tile * J.sstride + split) * TILE * TILE;
    float* outE = J.slab + ((size_t)((T - 1) * T / 2 + ti) * J.sstride + split) * TILE * TILE;
    auto store = [&](float* o, int bi, int bj, const floatx16& a) {
      put_partial(J, a, [&](int v) { return &o[(bi * 32 + acc_row(v, lane)) * TILE + bj * 32 + (lane & 31)]; });
    };
    if (wave == 0) {
      put(1, acc[1][0]);
      put(2, acc[1][1]);
    } else {
      put(0, acc[0][0]);
      put(3, acc[0][1]);
      put(4, acc4);
    }
    __syncthreads();
    if (wave == 0) {
      add(0, acc[0][0]);
      add(3, acc[0][1]);
      add(4, acc4);
      store(outD, 0, 0, acc[0][0]);
      store(outE, 0, 0, acc[0][1]);
      store(outE, 0, 1, acc4);
    } else {
      add(1, acc[1][0]);
      add(2, acc[1][1]);
      store(outD, 1, 0, acc[1][0]);
      store(outD, 1, 1, acc[1][1]);
    }
    return;
  }
  // wave w stores block row w: it hands the other block row's partials to the other
  // wave through LDS (the ring is free after the barrier), then adds the other
  // wave's.  Both sums are w0 + w1 (IEEE addition commutes): deterministic.
  __syncthreads();
  float* xo = lds;  // [wave][bj][16 values][64 lanes]
  float* out = J.slab + ((size_t)tile * J.sstride + split) * TILE * TILE;
  auto hand = [&](auto bic) {
    constexpr int bi = decltype(bic)::value;
#pragma unroll
    for (int bj = 0; bj < 2; ++bj)
      if (act[bi][bj])
#pragma unroll
        for (int v = 0; v < 16; ++v) xo[((wave * 2 + bj) * 16 + v) * 64 + lane] = acc[bi][bj][v];
  };
  auto keep = [&](auto bic) {
    constexpr int bi = decltype(bic)::value;
#pragma unroll
    for (int bj = 0; bj < 2; ++bj)
      if (act[bi][bj]) {
#pragma unroll
        for (int v = 0; v < 16; ++v) acc[bi][bj][v] += xo[(((1 - wave) * 2 + bj) * 16 + v) * 64 + lane];
        put_partial(J, acc[bi][bj],
                    [&](int v) { return &out[(bi * 32 + acc_row(v, lane)) * TILE + bj * 32 + (lane & 31)]; });
        // the slabs of the pair units' extra K-splits hold nothing of this tile: its
        // last full K-split writes them as zero partials
        if (split == sf - 1)
          for (int x = 1; x <= J.xsplits; ++x) {
            floatx16 z;
#pragma unroll
            for (int v = 0; v < 16; ++v) z[v] = 0.f;
            float* o = out + (size_t)x * TILE * TILE;
            put_partial(J, z, [&](int v) { return &o[(bi * 32 + acc_row(v, lane)) * TILE + bj * 32 + (lane & 31)]; });
          }
      }
  };
  if (wave == 0) hand(std::integral_constant<int, 1>{});
  else hand(std::integral_constant<int, 0>{});
  __syncthreads();
  if (wave == 0) keep(std::integral_constant<int, 0>{});
  else keep(std::integral_constant<int, 1>{});
}

// Every job of the launch is LDS-DMA-eligible or narrow (n <= 32: direct loads).
// 2 waves per SIMD (178 VGPRs): 4 workgroups per CU leave a 32-tile inversion
// workgroup (107 registers, 29 KB) room to run beside the pass
__global__ __launch_bounds__(X3_THREADS, 2) void kfac_factor_tiles_x3(FactorArgs args) {
  // (LDS only for the epilogue's hand-off: a block row, 16 KB; a pair's blocks, 20 KB)
  __shared__ __attribute__((aligned(16))) float lds[5 * 16 * 64];
  // (no start stagger here: the fp32 kernel's +2.5 % measured neutral on this one, MLP
  // line 1.951-1.954e8 without vs 1.951-1.957e8 with, 3 alternating runs, profiles/r06b/)
  const int task = xcd_task(blockIdx.x, gridDim.x);
  int j = 0;
  while (j + 1 < args.njobs && task >= args.task_end[j]) ++j;
  const int local = task - args.job[j].task_begin;
  const FactorJobDev& J = args.job[j];
  if (J.n <= 32)
    factor_task_narrow_direct<X3_NW>(J, args.segs, local, lds);
  else
    factor_task_x3<BK, 2>(J, args.segs, local, lds, args.split_major);
}


// ------------------------------------------------------------ conv operands
// Conv2d factors with each image staged whole in LDS (replaces the per-element
// register gather of the im2col / channel-major panel loaders for images that fit).
// F = sum_rows P[row]^T P[row], row = (image b, output position):
//   PATCH   (A, implicit F.unfold): P[(oh,ow)][(c,ki,kj)] = x_pad[b][c][oh*sh+ki][ow*sw+kj]
//   CHANNEL (G, permute(1,0,2,3)):  P[pos][c] = g[b][c][pos]
// A task is a group of blocks over WHOLE images.  Each image is
// staged into LDS once (coalesced loads of the next image in flight meanwhile);
// zero padding, the bias ones column and tile padding live in planes filled once
// per task.  An MFMA's k-lanes take different output ROWS (PATCH: oh = g*KR + k;
// CHANNEL: contiguous position segments), so along a row every lane's operand is
// one LDS read at base_lane + t*stride: no per-MFMA index arithmetic (stride 1:
// immediate offsets).  Rows past Ho read the A operand from the zero plane.
//   n <= 16 : one 16x16 block, v_mfma_f32_16x16x4f32 (KR = 4), the 4 waves take
//             different row groups / segments;
//   n <= 32 : one 32x32 quadrant, 32x32x2 (KR = 2), split over waves the same way;
//   else    : the lower triangle in 32x32 blocks, 4*CONV_CB per workgroup (CONV_CB
//             per wave, balanced to one block; each image staged once for all).
// Partials go to the slab / accumulator tiles exactly as the other paths (block
// (bi, bj) = quadrant (bi & 1, bj & 1) of tile (bi / 2, bj / 2)).
constexpr int CONV_LDS_MAX = 12288;  // staged floats per workgroup (48 KB of LDS)
constexpr int CONV_SRC_MAX = 2048;   // per-image staged elements (PATCH) / float4s (CHANNEL)

typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int CONV_CB = 2;  // 32x32 blocks per wave (mode 0): 4*CONV_CB per workgroup
// operand chunk of the two-block row loop: 2 steps ahead (4 MFMAs of 64 cycles cover the
// LDS latency) instead of 4 keeps the PATCH instances inside the 128-VGPR budget of 4
// workgroups per CU without spilling (LeNet-5: conv 2.90 vs 3.04 ms per pass, 1.69 vs
// 1.63e7 img/s, 3 alternating runs, profiles/r06b/)
constexpr int CONV_CK2 = 2;

struct ConvGeom {
  int mode;        // 0: 64x64 tiles, 1: narrow 32x32, 2: narrow 16x16
  int n;           // factor order
  int KR;          // k-lanes per MFMA (2 or 4)
  int B;           // images of the job: nseg batches x bseg images
  int bseg;        // images per batch (a multi-batch job walks the queued batches' bases)
  int T;           // MFMAs along one row group (PATCH: Wo; CHANNEL: segment length Q)
  int G;           // row groups (PATCH: ceil(Ho / KR)); CHANNEL: 1
  int stride;      // LDS step between consecutive MFMAs (PATCH: sw; CHANNEL: 1)
  int rowstep;     // PATCH: sh * Wp (one output row); CHANNEL: Q (one segment)
  int Ho;          // PATCH: output rows
  int plane;       // PATCH: Hp * Wp; CHANNEL: Lp = segments * Q (channel pitch)
  int Wp;          // PATCH: padded row pitch
  int ones_base;   // LDS offset of the all-ones plane (PATCH bias column)
  int zero_base;   // LDS offset of the all-zero plane (tile padding, rows past Ho)
  int lds;         // floats of LDS (>= the narrow reduce's 3 x 16 x 64)
  int src;         // staged source elements (PATCH) / float4s (CHANNEL) per image
  int nq;          // mode 0: 32x32 blocks of the factor's lower triangle
  int units;       // workgroups per K-split (mode 0: ceil(nq / (4*CONV_CB)) block groups; else 1)
  // mode 4 (kfac_factor_conv_x3: im2col operand split into bf16x3 in LDS)
  int nb;          // 32-blocks per factor edge (im2col rows padded to 32 nb)
  int L;           // output positions per image (Ho * Wo)
  int Wo, sh, sw;  // output row length, strides
  int LPC;         // positions per chunk (multiple of 16): an image is ceil(L / LPC) chunks
  int nch;         // chunks per image
  int pitch;       // bf16 elements per im2col row (LPC + 8: 16-byte reads conflict-free)
  int imgf;        // floats of one staged fp32 image (C padded planes)
  int ones;        // bias column (-1: none)
  int ldsb;        // bytes of dynamic LDS
  int kw;          // waves per block (nq <= 4: the block's k-steps interleaved over kw waves)
  // mode 5 (kfac_factor_conv_x3s: one 32 x 32 block from column-shifted image copies)
  int xs_ncopy;    // copies (C x kernel width), then the ones copy and the zero copy
  int xs_hp;       // rows per copy (padded image rows)
  int xs_pw;       // bf16 per copy row (>= 8 xs_g8)
  int xs_cs;       // bf16 per copy (>= xs_hp xs_pw)
  int xs_g8;       // 8-position groups per output row (ceil(Wo / 8): 1, 2, 4 or 8)
  int xs_grp;      // groups per image (Ho xs_g8, even); k-step t holds groups 2t, 2t + 1
  int xs_np;       // build slots per image (C xs_hp xs_wp2)
  int xs_wp2;      // build slots per padded row (ceil((W + 2 pw) / 2))
  // mode 6 (kfac_factor_conv_x3f: flattened column copies; xs_hp / xs_wp2 / xs_np too)
  int xf_nv;       // shifted variants per copy (8-byte fragment reads)
  int xf_vmap;     // kernel row ki's variant in bits 2ki .. 2ki+1
  int xf_one, xf_zero, xf_dummy;  // part byte offsets of the ones / zero copies, the dummy row
  int xf_nks;      // 16-position k-steps per image (ceil(L / 16))
  int xf_wave[4];  // multiplying wave w: pattern (bits 0-3) and F[q] (bits 4 + 3q ..)
  int xs_lb[32];   // block row m's fragment byte offset in a part (copy, row, column)
  int8_t xs_f[32]; // block row m's factor row / column (data, bias, padding rows n..31)
  // mode 6: copy (c, kj, v)'s part byte offset (shift included) in the u16 at 16 c + 2 kj + v
  int xf_cb[128];
};

constexpr int KFAC_CONV_OCC = 4;  // resident workgroups per CU the mode-0 instances are compiled for
template <int LAYOUT, int PMAXE, bool STRIDE1, int CB = CONV_CB, bool M3 = false>
__global__ __launch_bounds__(NTHREADS, (CB == 2 && !M3) ? KFAC_CONV_OCC : 4) void kfac_factor_conv(
    FactorArgs args, ConvGeom cg) {
  extern __shared__ __attribute__((aligned(16))) float cimg[];
  const int task = xcd_task(blockIdx.x, gridDim.x);
  int jx = 0;
  while (jx + 1 < args.njobs && task >= args.task_end[jx]) ++jx;
  const FactorJobDev& J = args.job[jx];
  const OpDev& op = J.x;
  const int local = task - J.task_begin;
  const int unit = local / J.splits, split = local - unit * J.splits;  // unit: block group
  // wave index through readfirstlane: the block bookkeeping derived from it (same[],
  // nmine, the row groups) is then wave-uniform (scalar branches, no exec-mask
  // juggling around the operand reads of the MFMA chain)
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // M3: the mode-3 instance (its three accumulators and operand rings stay out of the
  // other modes' register budget)
  const int mode = M3 ? 3 : cg.mode;
  const bool m16 = mode >= 2;  // 16x16x4 MFMA modes (2: one block; 3: blocks 00, 10, 11)
  const int klane = m16 ? lane >> 4 : lane >> 5;
  const int64_t b0 = (int64_t)split * cg.B / J.splits, b1 = (int64_t)(split + 1) * cg.B / J.splits;

  // staging map: source element (PATCH) / float4 (CHANNEL) q of this thread -> LDS index
  int dmap[PMAXE];
#pragma unroll
  for (int q = 0; q < PMAXE; ++q) {
    const int e = tid + q * NTHREADS;
    int d = -1;
    if (e < cg.src) {
      if (LAYOUT == KFAC_PATCH) {
        const int hw = op.H * op.W, c = e / hw, r = e - c * hw, h = r / op.W, w = r - h * op.W;
        d = c * cg.plane + (h + op.ph) * cg.Wp + (w + op.pw);
      } else {  // float index of the float4's first element (planes need not be 4-aligned)
        const int L4 = (int)op.L >> 2, c = e / L4;
        d = c * cg.plane + 4 * (e - c * L4);
      }
    }
    dmap[q] = d;
  }
  // next image in flight: PATCH stages single floats, CHANNEL float4s
  using PreT = std::conditional_t<LAYOUT == KFAC_PATCH, float, floatx4>;
  PreT pre[PMAXE];
  auto fetch = [&](int64_t b) {
    const int seg = (int)((uint32_t)b / (uint32_t)cg.bseg);
    const float* src = seg_base(J, args.segs, seg) + (b - (int64_t)seg * cg.bseg) * op.sB;
#pragma unroll
    for (int q = 0; q < PMAXE; ++q) {
      if (dmap[q] < 0) continue;
      if constexpr (LAYOUT == KFAC_PATCH) pre[q] = src[tid + q * NTHREADS];
      else pre[q] = reinterpret_cast<const floatx4*>(src)[tid + q * NTHREADS];
    }
  };
  auto commit = [&]() {
#pragma unroll
    for (int q = 0; q < PMAXE; ++q) {
      if (dmap[q] < 0) continue;
      if constexpr (LAYOUT == KFAC_PATCH) {
        cimg[dmap[q]] = pre[q];
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) cimg[dmap[q] + r] = pre[q][r];
      }
    }
  };

  // per-lane operand columns -> LDS offset of the column's plane position
  auto column = [&](int col) -> int {
    if (col >= op.cols) return (col == op.ones) ? cg.ones_base : cg.zero_base;
    if (LAYOUT == KFAC_PATCH) {
      const int kk = op.kh * op.kw, c = col / kk, r = col - c * kk, ki = r / op.kw;
      return c * cg.plane + ki * cg.Wp + (r - ki * op.kw);
    }
    return col * cg.plane;
  };
  // Blocks of this wave.  mode 0: the factor's lower triangle in 32x32 blocks
  // (b = tri index), 4*CB per workgroup (unit), block b = unit*4*CB + wave + 4i: the
  // workgroup stages each image once for all its blocks and the waves' shares differ
  // by at most one block.  Narrow modes: the one block, every wave.
  const int cl = m16 ? lane & 15 : lane & 31;
  int offA[CB], offB[CB], bij[CB];
  bool same[CB];
  int nmine = 0;
#pragma unroll
  for (int i = 0; i < CB; ++i) {
    const int bidx = unit * 4 * CB + wave + 4 * i;
    int bi = 0, bj = 0;
    if (mode == 0) tri_decode(bidx, bi, bj);
    const bool mine = mode ? i == 0 : bidx < cg.nq;
    nmine += mine;
    // mode 3: offA[0] / offA[1] = feature columns 0..15 / 16..31 (both operands)
    offA[i] = column(mode == 3 ? 16 * i + cl : 32 * bi + cl);
    offB[i] = column(32 * bj + cl);
    same[i] = bi == bj;
    bij[i] = (bi << 16) | bj;
  }

  floatx16 acc[CB];
  floatx4 acc16, acc16b, acc16c;  // mode 2: block 00; mode 3: blocks 00, 10, 11
#pragma unroll
  for (int i = 0; i < CB; ++i)
#pragma unroll
    for (int v = 0; v < 16; ++v) acc[i][v] = 0.f;
#pragma unroll
  for (int v = 0; v < 4; ++v) acc16[v] = acc16b[v] = acc16c[v] = 0.f;

  // one row group of one block: T MFMAs, operands read two MFMAs ahead (LDS latency
  // off the accumulator chain)
  // Operands in chunks of CK steps, double-buffered: chunk c+1's LDS reads are issued
  // before chunk c's MFMAs, so each read has CK MFMAs (>= 128 cycles) to land.  (B is
  // read even where it equals A -- a diagonal block: one more LDS read, but no select
  // that would make the next MFMA wait for the read.)
  auto row_mfmas = [&](const float* pa, const float* pb, bool, auto mfma) {
    constexpr int CK = 4;
    const int st = STRIDE1 ? 1 : cg.stride, T = cg.T, last = (T - 1) * st;
    float ca[CK], cb[CK], na[CK], nb[CK];
#pragma unroll
    for (int u = 0; u < CK; ++u) {
      const int o = min(u * st, last);
      ca[u] = pa[o];
      cb[u] = pb[o];
    }
    for (int t0 = 0; t0 < T; t0 += CK) {
#pragma unroll
      for (int u = 0; u < CK; ++u) {
        const int o = min((t0 + CK + u) * st, last);
        na[u] = pa[o];
        nb[u] = pb[o];
      }
#pragma unroll
      for (int u = 0; u < CK; ++u)
        if (t0 + u < T) mfma(ca[u], cb[u]);
#pragma unroll
      for (int u = 0; u < CK; ++u) {
        ca[u] = na[u];
        cb[u] = nb[u];
      }
    }
  };
  // two blocks (CB = 2) of one row group: operands for CK steps of both blocks per
  // chunk, double-buffered as in row_mfmas, MFMAs alternating between the blocks
  auto row_mfmas2 = [&](const float* pa0, const float* pb0, const float* pa1, const float* pb1) {
    constexpr int CK = CONV_CK2;
    const int st = STRIDE1 ? 1 : cg.stride, T = cg.T, last = (T - 1) * st;
    float ca[2][CK], cb[2][CK], na[2][CK], nb[2][CK];
#pragma unroll
    for (int u = 0; u < CK; ++u) {
      const int o = min(u * st, last);
      ca[0][u] = pa0[o]; cb[0][u] = pb0[o];
      ca[1][u] = pa1[o]; cb[1][u] = pb1[o];
    }
    for (int t0 = 0; t0 < T; t0 += CK) {
#pragma unroll
      for (int u = 0; u < CK; ++u) {
        const int o = min((t0 + CK + u) * st, last);
        na[0][u] = pa0[o]; nb[0][u] = pb0[o];
        na[1][u] = pa1[o]; nb[1][u] = pb1[o];
      }
#pragma unroll
      for (int u = 0; u < CK; ++u) {
        if (t0 + u < T) {
          acc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(ca[0][u], cb[0][u], acc[0], 0, 0, 0);
          acc[CB - 1] = __builtin_amdgcn_mfma_f32_32x32x2f32(ca[1][u], cb[1][u], acc[CB - 1], 0, 0, 0);
        }
      }
#pragma unroll
      for (int u = 0; u < CK; ++u) {
        ca[0][u] = na[0][u]; cb[0][u] = nb[0][u];
        ca[1][u] = na[1][u]; cb[1][u] = nb[1][u];
      }
    }
  };
  // mode 3: features 0..15 (v0) and 16..31 (v1) of CK steps per chunk, double-
  // buffered; each step feeds three 16x16x4 MFMAs (blocks 00 = v0 v0, 10 = v1 v0,
  // 11 = v1 v1): two LDS reads per three MFMAs, where the 32x32 block of mode 1 took
  // two per MFMA and computed the strictly-upper quarter too
  auto row_mfmas3 = [&](const float* p0, const float* p1) {
    constexpr int CK = 4;
    const int st = STRIDE1 ? 1 : cg.stride, T = cg.T, last = (T - 1) * st;
    float c0[CK], c1[CK], n0[CK], n1[CK];
#pragma unroll
    for (int u = 0; u < CK; ++u) {
      const int o = min(u * st, last);
      c0[u] = p0[o];
      c1[u] = p1[o];
    }
    for (int t0 = 0; t0 < T; t0 += CK) {
#pragma unroll
      for (int u = 0; u < CK; ++u) {
        const int o = min((t0 + CK + u) * st, last);
        n0[u] = p0[o];
        n1[u] = p1[o];
      }
#pragma unroll
      for (int u = 0; u < CK; ++u) {
        if (t0 + u < T) {
          acc16 = __builtin_amdgcn_mfma_f32_16x16x4f32(c0[u], c0[u], acc16, 0, 0, 0);
          acc16b = __builtin_amdgcn_mfma_f32_16x16x4f32(c1[u], c0[u], acc16b, 0, 0, 0);
          acc16c = __builtin_amdgcn_mfma_f32_16x16x4f32(c1[u], c1[u], acc16c, 0, 0, 0);
        }
      }
#pragma unroll
      for (int u = 0; u < CK; ++u) {
        c0[u] = n0[u];
        c1[u] = n1[u];
      }
    }
  };
  // one row group of every block of this wave (rowA / rowB: LDS offsets added to the
  // blocks' column offsets; zeroA: A read from the zero plane)
  auto blocks = [&](int rowA, int rowB, bool zeroA) {
    if constexpr (M3) {  // both operands from the same reads: a row past Ho reads zeros
      row_mfmas3(cimg + (zeroA ? cg.zero_base : offA[0] + rowA),
                 cimg + (zeroA ? cg.zero_base : offA[CB - 1] + rowA));
      return;
    }
    if (mode == 2) {
      row_mfmas(cimg + (zeroA ? cg.zero_base : offA[0] + rowA), cimg + offB[0] + rowB, true,
                [&](float a, float b) { acc16 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc16, 0, 0, 0); });
      return;
    }
    if constexpr (CB == 2) if (nmine == 2) {
      // both blocks in one pass, their MFMAs alternating (two independent chains)
      row_mfmas2(cimg + (zeroA ? cg.zero_base : offA[0] + rowA), cimg + offB[0] + rowB,
                 cimg + (zeroA ? cg.zero_base : offA[1] + rowA), cimg + offB[1] + rowB);
      return;
    }
#pragma unroll
    for (int i = 0; i < CB; ++i) {
      if (i >= nmine) break;
      row_mfmas(cimg + (zeroA ? cg.zero_base : offA[i] + rowA), cimg + offB[i] + rowB, same[i],
                [&](float a, float b) { acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[i], 0, 0, 0); });
    }
  };

  if (b0 < b1) fetch(b0);
  // constant planes (and the zero padding / segment tails of the image planes)
  for (int e = tid; e < cg.lds; e += NTHREADS)
    cimg[e] = (LAYOUT == KFAC_PATCH && e >= cg.ones_base && e < cg.zero_base) ? 1.f : 0.f;
  for (int64_t b = b0; b < b1; ++b) {
    __syncthreads();  // every wave done with the previous image (and the fill)
    commit();
    __syncthreads();
    if (b + 1 < b1) fetch(b + 1);  // next image's loads fly during the MFMAs
    if (nmine == 0) continue;
    if (LAYOUT == KFAC_PATCH) {
      for (int g = mode ? wave : 0; g < cg.G; g += mode ? 4 : 1) {
        const int oh = g * cg.KR + klane;  // rows past Ho: A from the zero plane
        blocks(oh * cg.rowstep, min(oh, cg.Ho - 1) * cg.rowstep, oh >= cg.Ho);
      }
    } else {
      const int sg = mode ? wave * cg.KR + klane : klane;
      blocks(sg * cg.rowstep, sg * cg.rowstep, false);
    }
  }

  float* out = J.slab + (size_t)split * TILE * TILE;  // narrow: tile 0
  if (mode == 1) {
    store_narrow(J, out, acc[0], cimg);
    return;
  }
  if constexpr (M3) {  // sum the 4 waves' three 16x16 partials in wave order (deterministic)
    __syncthreads();
    if (wave > 0) {
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        cimg[((wave - 1) * 12 + v) * 64 + lane] = acc16[v];
        cimg[((wave - 1) * 12 + 4 + v) * 64 + lane] = acc16b[v];
        cimg[((wave - 1) * 12 + 8 + v) * 64 + lane] = acc16c[v];
      }
    }
    __syncthreads();
    if (wave != 0) return;
    const int rr = (lane >> 4) * 4, cc = lane & 15;
#pragma unroll
    for (int blk = 0; blk < 3; ++blk) {
      const int bi = blk ? 1 : 0, bj = blk == 2 ? 1 : 0;
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        float t = blk == 0 ? acc16[v] : blk == 1 ? acc16b[v] : acc16c[v];
#pragma unroll
        for (int w = 0; w < 3; ++w) t += cimg[(w * 12 + blk * 4 + v) * 64 + lane];
        float* at = &out[(16 * bi + rr + v) * TILE + 16 * bj + cc];
        if (!J.accum) *at = t;
        else *at = J.sbeta == 0.f ? J.alpha * t : fmaf(J.sbeta, *at, J.alpha * t);
      }
    }
    return;
  }
  if (mode == 2) {  // sum the 4 waves' 16x16 partials in wave order (deterministic)
    __syncthreads();
    if (wave > 0) {
#pragma unroll
      for (int v = 0; v < 4; ++v) cimg[((wave - 1) * 4 + v) * 64 + lane] = acc16[v];
    }
    __syncthreads();
    if (wave != 0) return;
    // C/D map of 16x16x4: row = (lane >> 4) * 4 + v, col = lane & 15
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      float t = acc16[v];
#pragma unroll
      for (int w = 0; w < 3; ++w) t += cimg[(w * 4 + v) * 64 + lane];
      float* at = &out[((lane >> 4) * 4 + v) * TILE + (lane & 15)];
      if (!J.accum) *at = t;
      else *at = J.sbeta == 0.f ? J.alpha * t : fmaf(J.sbeta, *at, J.alpha * t);
    }
    return;
  }
  // block (bi, bj) = quadrant (bi & 1, bj & 1) of slab tile (bi / 2, bj / 2)
#pragma unroll
  for (int i = 0; i < CB; ++i) {
    if (i >= nmine) break;
    const int bi = bij[i] >> 16, bj = bij[i] & 0xffff, ti = bi >> 1, tj = bj >> 1;
    float* o = J.slab + ((size_t)(ti * (ti + 1) / 2 + tj) * J.sstride + split) * TILE * TILE +
               (bi & 1) * 32 * TILE + (bj & 1) * 32;
    put_partial(J, acc[i], [&](int v) { return &o[acc_row(v, lane) * TILE + (lane & 31)]; });
  }
}

// ------------------------------------------- conv factors in bf16x3 (mode 4)
// The im2col factor of a conv layer (PATCH operand, n > 32: LeNet-5's conv2 A, n = 151
// over 100 positions per image), F = sum over (image, position) P[pos]^T P[pos]
// (curvatures.py:341-343), on the bf16 MFMA at six products per fp32 product (the
// exact three-part split of the x3 / syrk3 kernels: 417 TF/s fp32-equivalent against
// the fp32 MFMA's 157).  One workgroup of 8 waves per CU takes whole images (a large
// image in chunks of LPC positions).  Per image it
//   * stages the fp32 image in LDS with its zero padding (the next image's loads fly
//     during the current one, its copy goes into the other of two image buffers);
//   * builds the explicit im2col in LDS, split ONCE into its three bf16 parts, laid out
//     [part][feature][position] with positions contiguous: an MFMA fragment -- 8
//     consecutive positions of one feature -- is one ds_read_b128 (row pitch LPC + 8
//     bf16: the 16-byte reads of a lane group hit distinct bank quads).  A thread owns
//     one 8-position group and every FS-th feature, so the lanes of a wave gather
//     consecutive features (neighbouring words; positions fastest gave 3-4-way bank
//     conflicts and 6 % more time, profiles/r06h/);
//   * multiplies: each wave its 32 x 32 blocks of the lower triangle (block b = wave +
//     8 i), six v_mfma_f32_32x32x16_bf16 per block and 16 positions, the next k-step's
//     fragments read during the current one's MFMAs.
// One im2col buffer (115 KB for conv2 A), so the build and the MFMAs of an image are
// two barrier-separated phases.  Tried: two buffers of half the positions with waves
// 0-3 building while waves 4-7 multiply (and the other way round): 389 vs 306 us per
// launch -- the 48-position chunks cost more per-chunk overhead than the overlap saved
// (profiles/r06g/).  Partials go to the slab tiles of the other conv paths.
constexpr bool CX3_PIPE = 1;
constexpr int CX3_THREADS = 512;
constexpr int CX3_WAVES = CX3_THREADS / 64;
constexpr int CX3_PM = CONV_SRC_MAX / CX3_THREADS;  // staged source elements per thread

template <int BPW>
__global__ __launch_bounds__(CX3_THREADS, 1) void kfac_factor_conv_x3(FactorArgs args, ConvGeom cg) {
  extern __shared__ __attribute__((aligned(16))) char cx3[];
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  const int task = xcd_task(blockIdx.x, gridDim.x);
  int jx = 0;
  while (jx + 1 < args.njobs && task >= args.task_end[jx]) ++jx;
  const FactorJobDev& J = args.job[jx];
  const OpDev& op = J.x;
  const int split = task - J.task_begin;  // one unit: task = split
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t b0 = (int64_t)split * cg.B / J.splits, b1 = (int64_t)(split + 1) * cg.B / J.splits;
  const int NR = 32 * cg.nb;              // im2col rows (features padded to 32 nb)
  const int partb = NR * cg.pitch * 2;    // bytes of one bf16 part
  char* colbuf = cx3;                     // [3][NR][pitch] bf16
  // two fp32 image buffers (imgf floats each), then a zero region of imgf floats: an
  // invalid position (past L) reads zero region + feature offset (< imgf)
  float* img = reinterpret_cast<float*>(cx3 + 3 * partb);
  int* posoff = reinterpret_cast<int*>(img + 3 * cg.imgf);  // nch * LPC positions (-1: past L)
  int* featoff = posoff + cg.nch * cg.LPC;                  // cols features
  // once per task: zero the im2col (padded feature rows, pitch slack) and the image
  // area (pad cells, zero region); the position and feature offset tables
  for (int e = tid; e < 3 * partb / 16; e += CX3_THREADS)
    reinterpret_cast<u32x4*>(colbuf)[e] = u32x4{0u, 0u, 0u, 0u};
  for (int e = tid; e < 3 * cg.imgf; e += CX3_THREADS) img[e] = 0.f;
  for (int q = tid; q < cg.nch * cg.LPC; q += CX3_THREADS) {
    const int oh = q / cg.Wo, ow = q - oh * cg.Wo;
    posoff[q] = q < cg.L ? oh * cg.sh * cg.Wp + ow * cg.sw : -1;
  }
  for (int f = tid; f < op.cols; f += CX3_THREADS) {
    const int kk = op.kh * op.kw, c = f / kk, r = f - c * kk, ki = r / op.kw, kj = r - ki * op.kw;
    featoff[f] = c * cg.plane + ki * cg.Wp + kj;
  }
  // staging map of this thread's source elements (image (c, h, w) -> padded plane)
  int dmap[CX3_PM];
#pragma unroll
  for (int q = 0; q < CX3_PM; ++q) {
    const int e = tid + q * CX3_THREADS;
    int d = -1;
    if (e < cg.src) {
      const int hw = op.H * op.W, c = e / hw, r = e - c * hw, h = r / op.W, w = r - h * op.W;
      d = c * cg.plane + (h + op.ph) * cg.Wp + (w + op.pw);
    }
    dmap[q] = d;
  }
  float pre[CX3_PM];
  auto fetch = [&](int64_t b) {
    const int seg = (int)((uint32_t)b / (uint32_t)cg.bseg);
    const float* src = seg_base(J, args.segs, seg) + (b - (int64_t)seg * cg.bseg) * op.sB;
#pragma unroll
    for (int q = 0; q < CX3_PM; ++q)
      if (dmap[q] >= 0) pre[q] = src[tid + q * CX3_THREADS];
  };
  auto commit = [&](int buf) {
#pragma unroll
    for (int q = 0; q < CX3_PM; ++q)
      if (dmap[q] >= 0) img[buf + dmap[q]] = pre[q];
  };
  // this wave's blocks of the lower triangle and its lanes' fragment offsets: blocks
  // wave + 8 i, or (few blocks, kw > 1) block wave / kw over every kw-th k-step
  const int m = lane & 31, hh = lane >> 5;
  const int KW = cg.kw, kp = wave % KW;
  auto block_of = [&](int i) { return KW > 1 ? wave / KW : wave + CX3_WAVES * i; };
  int offA[BPW], offB[BPW];
  bool diag[BPW];
  int nmine = 0;
#pragma unroll
  for (int i = 0; i < BPW; ++i) {
    const int b = block_of(i);
    int bi = 0, bj = 0;
    if (b < cg.nq && (KW == 1 || i == 0)) {
      tri_decode(b, bi, bj);
      ++nmine;
    }
    offA[i] = ((32 * bi + m) * cg.pitch + 8 * hh) * 2;
    offB[i] = ((32 * bj + m) * cg.pitch + 8 * hh) * 2;
    diag[i] = bi == bj;
  }
  floatx16 acc[BPW];
#pragma unroll
  for (int i = 0; i < BPW; ++i)
#pragma unroll
    for (int v = 0; v < 16; ++v) acc[i][v] = 0.f;

  // build chunk c of the image in fp32 buffer `buf` into im2col buffer `col`.  Thread t
  // owns the 8-position group g = t / FS of the chunk and features fi, fi + FS, ...
  // (fi = t % FS, FS = 512 / (LPC / 8)): lanes of a wave take consecutive FEATURES of
  // one group, so their fp32 gathers hit neighbouring words; the group's positions are
  // resolved once per chunk.  Only the k-steps holding valid positions are built (a
  // short last chunk builds few: the groups its MFMAs read, past-L positions as zeros --
  // the buffer still holds an earlier chunk beyond them).
  const int FS = CX3_THREADS / (cg.LPC / 8);
  const int g = tid / FS, fi = tid - g * FS;
  auto build = [&](char* col, int buf, int c) {
    const int valid_pos = min(cg.LPC, cg.L - c * cg.LPC);
    const int groups = 2 * ((valid_pos + 15) / 16);
    if (g >= groups) return;
    const int q0 = c * cg.LPC + 8 * g;
    int po[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int pq = posoff[q0 + e];
      po[e] = pq >= 0 ? buf + pq : 2 * cg.imgf;
    }
    char* dstg = col + 16 * g;
    for (int f = fi; f < op.cols; f += FS) {
      const int fo = featoff[f];
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = img[po[e] + fo];
      const X3Frag fr = x3_split8(v);
      char* dst = dstg + f * cg.pitch * 2;
#pragma unroll
      for (int p = 0; p < 3; ++p) *reinterpret_cast<bf16x8*>(dst + p * partb) = fr.p[p];
    }
    // the bias ones column: 1 on the chunk's valid positions, 0 past them
    if (cg.ones >= 0 && fi == FS - 1) {
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = 8 * g + e < valid_pos ? 1.f : 0.f;
      const X3Frag fr = x3_split8(v);
      char* dst = dstg + cg.ones * cg.pitch * 2;
#pragma unroll
      for (int p = 0; p < 3; ++p) *reinterpret_cast<bf16x8*>(dst + p * partb) = fr.p[p];
    }
  };
  auto frag = [&](const char* col, int off, X3Frag& fr) __attribute__((always_inline)) {
#pragma unroll
    for (int p = 0; p < 3; ++p) fr.p[p] = *reinterpret_cast<const bf16x8*>(col + p * partb + off);
  };
  // the fragments of k-step s of every block slot of the wave, unconditionally: a
  // diagonal block reads its A twice, a slot past the wave's blocks block (0, 0), and its
  // MFMAs go to an accumulator never stored (a conditional read made the compiler wait
  // lgkmcnt(0) in front of every block's MFMAs)
  struct KStep {
    X3Frag A[BPW], B[BPW];
  };
  auto load_step = [&](const char* col, int s, KStep& k) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < BPW; ++i) {
      frag(col, offA[i] + 32 * s, k.A[i]);
      frag(col, offB[i] + 32 * s, k.B[i]);
    }
  };
  auto mul_step = [&](const KStep& k) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < BPW; ++i) x3_six(acc[i], k.A[i], k.B[i]);
  };
  // k-steps of chunk c, software-pipelined two deep where the registers allow: step
  // s + 1's LDS reads are in flight during step s's MFMAs (scheduling fences: left alone
  // the compiler sinks the prefetch behind the MFMAs; past the last k-step the prefetch
  // reloads it, unconditionally)
  auto mma = [&](const char* col, int c) __attribute__((always_inline)) {
    const int kst = (min(cg.LPC, cg.L - c * cg.LPC) + 15) / 16;  // 16-position k-steps
    if constexpr (BPW > 2 || !CX3_PIPE) {  // (two steps of 3 blocks in registers spill)
      for (int s = kp; s < kst; s += KW) {
        KStep k;
        load_step(col, s, k);
        mul_step(k);
      }
      return;
    }
    // this wave's k-steps kp + j kw, j < J
    const int J = kp < kst ? (kst - kp + KW - 1) / KW : 0;
    if (J == 0) return;
    KStep k0, k1;
    load_step(col, kp, k0);
    int j = 0;
    for (; j + 2 <= J; j += 2) {
      load_step(col, kp + (j + 1) * KW, k1);
      __builtin_amdgcn_sched_barrier(0);
      mul_step(k0);
      __builtin_amdgcn_sched_barrier(0);
      load_step(col, kp + min(j + 2, J - 1) * KW, k0);
      __builtin_amdgcn_sched_barrier(0);
      mul_step(k1);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (j < J) mul_step(k0);
  };

  // per image (and chunk of its positions): build the im2col, barrier, multiply,
  // barrier; the next image's loads fly during the current one and its fp32 copy goes
  // into the other image buffer (last read by the previous image's builds)
  if (b0 < b1) fetch(b0);
  __syncthreads();  // (the zero fill and the tables before the first commit)
  if (b0 < b1) commit(0);
  for (int64_t b = b0; b < b1; ++b) {
    const int buf = (int)((b - b0) & 1) * cg.imgf;
    for (int c = 0; c < cg.nch; ++c) {
      __syncthreads();  // image b committed; every wave done reading the previous im2col
      if (c == 0 && b + 1 < b1) fetch(b + 1);
      build(colbuf, buf, c);
      __syncthreads();
      if (c == cg.nch - 1 && b + 1 < b1) commit(cg.imgf - buf);
      mma(colbuf, c);
    }
  }
  __syncthreads();  // (every wave's last MFMA reads before the partial-sum exchange)
  // block (bi, bj) = quadrant (bi & 1, bj & 1) of slab tile (bi / 2, bj / 2)
  auto at = [&](int i, int v) __attribute__((always_inline)) {
    int bi, bj;
    tri_decode(block_of(i), bi, bj);
    const int ti = bi >> 1, tj = bj >> 1;
    float* o = J.slab + ((size_t)(ti * (ti + 1) / 2 + tj) * J.sstride + split) * TILE * TILE +
               (bi & 1) * 32 * TILE + (bj & 1) * 32;
    return &o[acc_row(v, lane) * TILE + (lane & 31)];
  };
  float old[BPW][16];
  if (kp == 0) load_partials(J, nmine, old, at);  // (in flight across the exchange)
  // kw > 1: the kw partial sums of a block meet in LDS (the im2col buffers are free
  // after the last barrier), summed in wave order by its first wave (deterministic)
  if (KW > 1) {
    float* red = reinterpret_cast<float*>(colbuf);
    if (kp > 0 && nmine)
#pragma unroll
      for (int v = 0; v < 16; ++v) red[(wave * 16 + v) * 64 + lane] = acc[0][v];
    __syncthreads();
    if (kp > 0) return;
    for (int w = wave + 1; w < wave + KW; ++w)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[0][v] += red[(w * 16 + v) * 64 + lane];
  }
  put_partials(J, nmine, acc, old, at);
}

// ------------------------------- one-block conv factors in bf16x3 (mode 5)
// The im2col factor of a conv layer with 17 <= n <= 32 (LeNet-5's conv1 A: 26 over 784
// positions per image, curvatures.py:341-343) as ONE 32 x 32 block, on the bf16 MFMA.
// An explicit im2col of 784 positions costs more to build than its MFMAs (mode 4 measured
// 313 vs 139 us for the fp32 mode 3).  Here no im2col is built: the MFMA fragment of
// feature (c, ki, kj) at output positions (oh, ow0 .. ow0 + 7) is row oh sh + ki,
// columns ow0 .. ow0 + 7 of a COLUMN COPY (c, kj) of the padded image,
//   copy(c, kj)[r][ow] = padded[c][r][ow sw + kj]   (0 for ow >= Wo),
// so the C x kw copies, split once per entry into bf16 hi / mid / lo, hold every
// fragment as one ds_read_b128 (kh x fewer entries than the im2col).  A k-step is 16
// positions: lanes 0-31 read group 2t, lanes 32-63 group 2t + 1 (8 positions of one
// output row each; rows padded to 8 ceil(Wo / 8) positions, the padding zero in every
// copy).  The bias row reads a ones copy, rows past n a zero copy.  A = B (one diagonal
// block): six MFMAs per k-step on one fragment triple.
// One workgroup of 8 waves per CU, two copy buffers, in two groups of 4 waves (one per
// SIMD each) that swap roles every image: in phase i group i mod 2 multiplies image i
// (its 4 waves take k-steps wave + 4 j, fragments two k-steps ahead) while the other
// group builds image i + 1 into the other buffer and then issues the loads of its next
// image (i + 3: a whole phase to land; buffer loads whose out-of-image offsets return
// 0); one barrier per phase.  The build splits each image element ONCE and writes it to
// the kw copies that hold it.  The 8 partial sums meet in LDS in wave order.  The host
// deals factor rows to block rows so the 16 lanes of each ds_read_b128 group read 16
// distinct bank quads.
// Measured on the LeNet-5 pass (conv1 A, 60,000 images; profiles/r06k-r06r): the fp32
// mode 3 0.685 ms; this kernel 0.47 (MFMA phases alone 0.45, builds alone 0.27).  On
// the way: one LDS table read per k-step that the fragment addresses waited on, a
// register mask of odd group counts that waited on the prefetched reads, a conditional
// prefetch (lgkmcnt(0)), a phase loop whose branch split the in-flight loads' live
// ranges (vmcnt waits in the MFMA loop), lambdas not inlined (the kernel arguments
// copied to scratch) and a build that split every copy entry (kw x the VALU) each
// held it at 0.53-0.69 ms; 8 waves building after their MFMAs 0.67; two 4-wave
// workgroups per CU with a buffer each 0.67 (their phases stay in step).
constexpr int XS_THREADS = 512;
constexpr int XS_WAVES = XS_THREADS / 64;
constexpr int XS_GROUP = XS_THREADS / 2;  // threads per role group
constexpr int XS_SP = 4;                  // build slots per group thread and image (<= 1024)
constexpr int XS_KW = 8;                  // kernel width at most
constexpr int XS_LDS_MAX = 134144;        // (as mode 4: a 29 KB inversion workgroup still fits beside it)
constexpr int XS_ZPAD = 256;              // zero bytes after the zero copy: padding rows' column offsets
constexpr int XS_DUMMY = 16;              // (alignment slack after each part)

// the copy (k) and row offset of block row m (feature m; the bias row; padding rows)
__host__ __device__ inline void xs_lane(int m, int cols, int ones, int kh, int kw, int ncopy, int& k, int& row) {
  if (m < cols) {
    const int kk = kh * kw, c = m / kk, r = m - c * kk, ki = r / kw;
    k = c * kw + (r - ki * kw);
    row = ki;
  } else if (m == ones) {
    k = ncopy;
    row = 0;
  } else {  // (rows < kh: a read stays inside the zero copy)
    k = ncopy + 1;
    row = (m - cols) % kh;
  }
}

__global__ __launch_bounds__(XS_THREADS, 1) void kfac_factor_conv_x3s(FactorArgs args, ConvGeom cg) {
  extern __shared__ __attribute__((aligned(16))) char cxs[];
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  const int task = xcd_task(blockIdx.x, gridDim.x);
  int jx = 0;
  while (jx + 1 < args.njobs && task >= args.task_end[jx]) ++jx;
  const FactorJobDev& J = args.job[jx];
  const OpDev& op = J.x;
  const int split = task - J.task_begin;  // one unit: task = split
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t b0 = (int64_t)split * cg.B / J.splits, b1 = (int64_t)(split + 1) * cg.B / J.splits;
  // two buffers of [part][copy][row][ow] (copies (c, kj), the ones copy, the zero copy
  // and its pad)
  const int partb = (cg.xs_ncopy + 2) * cg.xs_cs * 2 + XS_ZPAD + XS_DUMMY;
  const int bufb = 3 * partb;
  // once per task: zero both buffers (padding, out-of-image entries and the zero copy
  // are never written again), then the ones copies' hi parts
  for (int e = tid; e < 2 * bufb / 16; e += XS_THREADS)
    reinterpret_cast<u32x4*>(cxs)[e] = u32x4{0u, 0u, 0u, 0u};
  __syncthreads();
  // (the rows oh sh the bias row reads)
  const int Ho = cg.L / cg.Wo;
  if (cg.ones >= 0)
    for (int e = tid; e < 2 * Ho * cg.Wo; e += XS_THREADS) {
      const int bs = e / (Ho * cg.Wo), r = e - bs * Ho * cg.Wo, h = r / cg.Wo;
      *reinterpret_cast<uint16_t*>(cxs + bs * bufb +
                                   (cg.xs_ncopy * cg.xs_cs + h * cg.sh * cg.xs_pw + (r - h * cg.Wo)) * 2) = 0x3f80;
    }
  // The build, per image element once: thread slot (c, r, col) (col even, padded
  // coordinates, stride 1) loads elements col .. col + 2 of padded row r of channel c,
  // splits the pairs (col, col + 1) and (col + 1, col + 2) and writes them to every copy
  // (c, kj) holding them at an even output column: ow = col - kj (kj even) or
  // col + 1 - kj (kj odd), when 0 <= ow < Wo (Wo even: a pair is wholly in or out).
  // Its source byte offsets (outside the image: past the buffer record, loads return
  // 0), the byte offset of (copy (c, 0), row r, column col) and the mask of kj written.
  constexpr int OUT = 0x7ffffff0;
  const int wp2 = cg.xs_wp2, rowp = cg.xs_hp * wp2;
  int sx[XS_SP][3], dbase[XS_SP], kmask[XS_SP];
  const int gt = tid % XS_GROUP, grp = wave / (XS_WAVES / 2);  // (both groups build every slot)
  const int nsp = (cg.xs_np + XS_GROUP - 1) / XS_GROUP;          // slots per thread (uniform)
#pragma unroll
  for (int i = 0; i < XS_SP; ++i) {
    const int e = gt + i * XS_GROUP;
    sx[i][0] = sx[i][1] = sx[i][2] = OUT;
    dbase[i] = 0;
    kmask[i] = 0;
    if (e < cg.xs_np) {
      const int c = e / rowp, rem = e - c * rowp, r = rem / wp2, col = 2 * (rem - r * wp2);
      const int h = r - op.ph;
#pragma unroll
      for (int d = 0; d < 3; ++d) {
        const int w = col + d - op.pw;
        if (h >= 0 && h < op.H && w >= 0 && w < op.W) sx[i][d] = ((c * op.H + h) * op.W + w) * 4;
      }
      dbase[i] = (c * op.kw * cg.xs_cs + r * cg.xs_pw + col) * 2;
      for (int kj = 0; kj < op.kw; ++kj) {
        const int ow = col - kj + (kj & 1);
        if (ow >= 0 && ow < cg.Wo) kmask[i] |= 1 << kj;
      }
    }
  }
  const int irec = op.C * op.H * op.W * 4;  // bytes of one image
  float v0[XS_SP][3];
  auto fetch = [&](int64_t b) __attribute__((always_inline)) {
    const int seg = (int)((uint32_t)b / (uint32_t)cg.bseg);
    const float* src = seg_base(J, args.segs, seg) + (b - (int64_t)seg * cg.bseg) * op.sB;
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(src), 0, irec, 0x00020000);
#pragma unroll
    for (int i = 0; i < XS_SP; ++i) {
      if (i >= nsp) break;
#pragma unroll
      for (int d = 0; d < 3; ++d)
        v0[i][d] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, sx[i][d], 0, 0));
    }
  };
  const int kstep = cg.xs_cs * 2 - 2;  // byte step of (copy kj, column col - kj) per kj
  auto build = [&](char* buf) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < XS_SP; ++i) {
      if (i >= nsp) break;
      uint32_t p0[3], p1[3];
      split3(v0[i][0], v0[i][1], p0[0], p0[1], p0[2]);
      split3(v0[i][1], v0[i][2], p1[0], p1[1], p1[2]);
#pragma unroll
      for (int kj = 0; kj < XS_KW; ++kj) {
        if (kj >= op.kw) break;
        if (kmask[i] >> kj & 1) {
          char* d = buf + dbase[i] + kj * kstep + 2 * (kj & 1);
#pragma unroll
          for (int q = 0; q < 3; ++q)
            *reinterpret_cast<uint32_t*>(d + q * partb) = (kj & 1) ? p1[q] : p0[q];
        }
      }
    }
  };
  // this lane's block row (the host's assignment of factor rows to block rows: lanes
  // of one ds_read_b128 group on distinct bank quads); lanes 32-63 take the odd groups
  // (tables read with constant indices only: a lane-indexed read of the by-value
  // argument copies the kernel arguments to scratch and reloads fields from there)
  const int hi = lane >> 5;
  int lbase = 0, fme = 0;
#pragma unroll
  for (int t = 0; t < 32; ++t) {
    int e = cg.xs_lb[t], f = cg.xs_f[t];
    asm volatile("" : "+s"(e), "+s"(f));  // (opaque: no select of addresses)
    lbase = (lane & 31) == t ? e : lbase;
    fme = tid == t ? f : fme;
  }
  __shared__ int ftab[32];  // block row -> factor row / column (the epilogue's stores)
  if (tid < 32) ftab[tid] = fme;
  floatx16 acc, acc2;  // (hh + mm, and the cross products' half: x3_four)
#pragma unroll
  for (int v = 0; v < 16; ++v) acc[v] = acc2[v] = 0.f;
  // group q = 2t + hi of k-step t: output row q / g8, columns 8 (q mod g8) .. + 7.  A
  // wave's k-steps t = gw + 4 j are groups q0 + 8 j, and g8 divides 8, so its fragment
  // addresses are a0 + j delta (no per-k-step index math; a table read in LDS, which the
  // addresses waited on, put its latency in front of every k-step's MFMAs).  The group
  // count is even (host), so every k-step holds two real groups.
  constexpr int GW = XS_WAVES / 2;
  const int nks = cg.xs_grp / 2, gw = wave % GW;
  const int Jn = gw < nks ? (nks - gw + GW - 1) / GW : 0;
  const int q0 = 2 * gw + hi, oh0 = q0 / cg.xs_g8;
  const int a0 = lbase + oh0 * cg.sh * cg.xs_pw * 2 + 16 * (q0 - oh0 * cg.xs_g8);
  const int delta = (8 / cg.xs_g8) * cg.sh * cg.xs_pw * 2;
  auto load = [&](const char* buf, int j, X3Frag& fr) __attribute__((always_inline)) {
    const char* p = buf + a0 + j * delta;
#pragma unroll
    for (int r = 0; r < 3; ++r) fr.p[r] = *reinterpret_cast<const bf16x8*>(p + r * partb);
  };
  // this wave's k-steps of an image (gw: its index in the group), the next one's reads
  // in flight during the current one's MFMAs
  auto mma = [&](const char* buf) __attribute__((always_inline)) {
    if (Jn == 0) return;
    // (scheduling fences: left alone the compiler sinks each prefetch behind the MFMAs
    // of the fragments whose registers it reuses, and every k-step waits for its reads;
    // the loads are unconditional -- past the last k-step a harmless reload -- since a
    // conditional load made the next wait lgkmcnt(0))
    const int last = Jn - 1;
    X3Frag k0, k1, k2;
    load(buf, 0, k0);
    load(buf, min(1, last), k1);
    int j = 0;
    for (; j + 3 <= Jn; j += 3) {
      load(buf, min(j + 2, last), k2);
      __builtin_amdgcn_sched_barrier(0);
      x3_four(acc, acc2, k0);
      __builtin_amdgcn_sched_barrier(0);
      load(buf, min(j + 3, last), k0);
      __builtin_amdgcn_sched_barrier(0);
      x3_four(acc, acc2, k1);
      __builtin_amdgcn_sched_barrier(0);
      load(buf, min(j + 4, last), k1);
      __builtin_amdgcn_sched_barrier(0);
      x3_four(acc, acc2, k2);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (j < Jn) x3_four(acc, acc2, k0);
    if (j + 1 < Jn) x3_four(acc, acc2, k1);
  };

  // phase i: group i % 2 multiplies image i, the other group builds image i + 1, then
  // loads image i + 3 (its next build); group 0 builds image 0 first.  One code path per
  // group, each phase pair straight-line: with one loop and a branch per phase the
  // compiler gave the in-flight loads the fragment registers (live ranges split at the
  // branch), and loads in flight on any path into a loop head (the other group's
  // prologue, this group's own) made it wait on them inside every multiply phase
  const int64_t nimg = b1 - b0;
  auto phase_mma = [&](int64_t i) __attribute__((always_inline)) {
    if (i < nimg) mma(cxs + (int)(i & 1) * bufb);
    __syncthreads();
  };
  auto phase_build = [&](int64_t i) __attribute__((always_inline)) {
    if (i + 1 < nimg) {
      build(cxs + (int)((i + 1) & 1) * bufb);
      if (i + 3 < nimg) fetch(b0 + i + 3);
    }
    __syncthreads();
  };
  if (grp == 0) {
    if (nimg > 0) {
      fetch(b0);
      build(cxs);
      if (nimg > 2) {
        fetch(b0 + 2);
#pragma unroll
        for (int i = 0; i < XS_SP; ++i) asm volatile("" ::"v"(v0[i][0]), "v"(v0[i][1]), "v"(v0[i][2]));  // (landed)
      }
    }
    __syncthreads();
    for (int64_t i = 0; i < nimg; i += 2) {
      phase_mma(i);
      phase_build(i + 1);
    }
  } else {
    if (nimg > 1) fetch(b0 + 1);
    __syncthreads();
    for (int64_t i = 0; i < nimg; i += 2) {
      phase_build(i);
      phase_mma(i + 1);
    }
  }
  // the 8 waves' partial sums, summed in wave order by wave 0 (deterministic); then
  // acc + acc2 + acc2^T, the transpose through LDS (wave 0's LDS operations complete in
  // order: its writes are read back with no barrier)
  float* red = reinterpret_cast<float*>(cxs);
  float* red2 = red + (XS_WAVES - 1) * 16 * 64;
  if (wave > 0)
#pragma unroll
    for (int v = 0; v < 16; ++v) {
      red[((wave - 1) * 16 + v) * 64 + lane] = acc[v];
      red2[((wave - 1) * 16 + v) * 64 + lane] = acc2[v];
    }
  __syncthreads();
  if (wave > 0) return;
  for (int w = 0; w < XS_WAVES - 1; ++w)
#pragma unroll
    for (int v = 0; v < 16; ++v) {
      acc[v] += red[(w * 16 + v) * 64 + lane];
      acc2[v] += red2[(w * 16 + v) * 64 + lane];
    }
  float* tr = red2 + (XS_WAVES - 1) * 16 * 64;  // 32 x 33
#pragma unroll
  for (int v = 0; v < 16; ++v) tr[acc_row(v, lane) * 33 + (lane & 31)] = acc2[v];
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
  for (int v = 0; v < 16; ++v) acc[v] += acc2[v] + tr[(lane & 31) * 33 + acc_row(v, lane)];
  float* o = J.slab + (size_t)split * TILE * TILE;  // block (0, 0) of slab tile 0
  const int fc = ftab[lane & 31];
  put_partial(J, acc, [&](int v) { return &o[ftab[acc_row(v, lane)] * TILE + fc]; });
}

// ------------------------- conv factors from flattened column copies (mode 6)
// The im2col factor of a stride-1 conv layer with 32 < n <= 160 (LeNet-5's conv2 A: 151
// features over 100 positions per image, curvatures.py:341-343) without an im2col.
// With the output positions flattened, p = oh Wo + ow, the patch entry of feature
// (c, ki, kj) at p is padded[c][oh + ki][ow + kj] = copy(c, kj)[ki Wo + p], where
//   copy(c, kj)[r Wo + ow] = padded[c][r][ow + kj]      (r < Hp, ow < Wo)
// is the padded image's column window of width Wo, rows kept at pitch Wo.  So C x kw
// copies (kh x fewer entries than the im2col, 25 KB per LeNet-5 image in three bf16
// parts instead of 102 KB) hold every MFMA fragment -- 8 consecutive positions of one
// feature -- at element ki Wo + p.  8-byte reads need ki Wo + shift = 0 mod 4: each copy
// is kept in NV <= 2 variants shifted by the residues the kernel rows need (LeNet-5
// conv2, Wo = 10: shifts 0 and 2).  Positions past L in the last 16-position k-step
// read the next rows' data, so that k-step's fragments are masked.  The bias row reads
// a ones copy, padding rows a zero copy.
// Copy placement (host, conv_x3f_geom): every copy (c, kj, v) has its own base, chosen so
// the 8-byte fragment reads of each 16-lane group hit 16 distinct bank pairs (a search
// over the bases' residues mod 128 B; a uniform copy stride left 2-way conflicts on 8 of
// LeNet-5's 10 groups: the reads took twice their time, `profiles/r06z4/`).  The bases
// sit in an LDS table (xf_cb, 16 entries per channel).
// As in mode 5: one workgroup of 8 waves per CU, two copy buffers, two groups of 4
// waves that swap roles every image (one multiplies image i, the other builds image
// i + 1 and loads image i + 3).  The build works from per-slot records made once per
// task (source offsets, destination offset, kernel columns in range): recomputing the
// slot geometry per image (integer divisions) and a branch per copy made the build the
// bound (3.9 us per image against 3.6 us of MFMAs; 425 VALU, 104 branches per wave).
constexpr int XF_THREADS = 512;
constexpr int XF_WAVES = XF_THREADS / 64;
constexpr int XF_GROUP = XF_THREADS / 2;  // threads per role group
constexpr int XF_GW = XF_WAVES / 2;       // waves per role group
constexpr int XF_SP = 3;                  // build slots per group thread and image (<= 768)
constexpr int XF_BPW = 4;                 // blocks per multiplying wave (nq <= 16)
constexpr int XF_KW = 8;                  // kernel width at most
constexpr int XF_CB = 256;                // copy-base table entries (C x 2 XF_KW: C <= 16)
constexpr int XF_PART = 19456;            // bytes per part (copies, ones, zero, dummy)
constexpr int XF_BUF = 3 * XF_PART;       // one copy buffer (hi, mid, lo parts)
constexpr int XF_REC = 2 * XF_BUF;        // build-slot records: [slot i][group thread] u32x2
constexpr int XF_TBL = XF_REC + XF_SP * XF_GROUP * 8;  // copy bases: u16 [c][kj][v] (v < 2)
constexpr int XF_LDS = XF_TBL + XF_CB * 2;  // (a 29 KB inversion workgroup still fits beside it)
static_assert(XF_LDS <= 134144, "x3f LDS");

// A multiplying wave's blocks as pairs (a, b) of indices into its fragment set F: block
// (F[a], F[b]); a diagonal block (a = b) takes x3_four (four MFMAs and a transposed
// half, acc2) instead of six.  Assignments (conv_x3f_geom), from an exact-cover search
// over the lower triangle's blocks (<= 4 blocks and <= 4 fragments per wave, block order
// maximizing the MFMAs between a fragment's reload and its next use):
//   5 block rows (n = 129..160): F = {0,1,2,3} (0,0) (1,1) (3,2) -- 14 MFMAs per k-step;
//     {0,1,2,4} (2,2) (2,0) (1,0) (4,1); {1,2,3,4} (2,1) (3,1) (4,3) (4,4);
//     {0,2,3,4} (3,3) (3,0) (4,0) (4,2) -- 22 each (six-product diagonals: 24 on the
//     busiest wave), >= 8 MFMAs of slack per reload (was 6);
//   4 block rows (97..128): F = {0,1,2,3} for all: (0,0) (1,1) (3,2); (1,0) (2,2) (3,3);
//     (2,0) (3,1); (2,1) (3,0) -- 14, 14, 12, 12.
struct XfPat {
  int a[4], b[4], n;
};
constexpr XfPat XF_PAT[] = {
    {{0, 1, 3, 0}, {0, 1, 2, 0}, 3}, {{2, 2, 1, 3}, {2, 0, 0, 1}, 4}, {{1, 2, 3, 3}, {0, 0, 2, 3}, 4},
    {{2, 2, 3, 3}, {2, 0, 0, 1}, 4}, {{1, 2, 3, 0}, {0, 2, 3, 0}, 3}, {{2, 3, 0, 0}, {0, 1, 0, 0}, 2},
    {{2, 3, 0, 0}, {1, 0, 0, 0}, 2}};
constexpr int XF_NPAT = sizeof(XF_PAT) / sizeof(XF_PAT[0]);
constexpr int XF_D2 = 2;  // diagonal blocks per wave at most (acc2 sets)
// (the epilogue's exchange -- 4 waves x 6 sets of 16 x 64 floats -- and 4 transpose tiles
// fit the two copy buffers)
static_assert(2 * XF_BUF >= (XF_GW * (XF_BPW + XF_D2) * 16 * 64 + XF_GW * 32 * 33) * 4, "x3f epilogue LDS");
__host__ __device__ constexpr int xf_pat_frags(const XfPat& p) {
  int m = 0;
  for (int s = 0; s < p.n; ++s) m = std::max(m, std::max(p.a[s], p.b[s]) + 1);
  return m;
}
__host__ __device__ constexpr int xf_pat_last_use(const XfPat& p, int q) {
  int l = -1;
  for (int s = 0; s < p.n; ++s)
    if (p.a[s] == q || p.b[s] == q) l = s;
  return l;
}
__host__ __device__ constexpr int xf_pat_diag(const XfPat& p, int s) {  // acc2 set of block s
  int d = 0;
  for (int t = 0; t < s; ++t) d += p.a[t] == p.b[t];
  return d;
}
__host__ __device__ inline int xf_pat_blocks(int pat) { return XF_PAT[pat].n; }
__host__ __device__ inline int xf_pat_a(int pat, int s) { return XF_PAT[pat].a[s]; }
__host__ __device__ inline int xf_pat_b(int pat, int s) { return XF_PAT[pat].b[s]; }

__global__ __launch_bounds__(XF_THREADS, 1) void kfac_factor_conv_x3f(FactorArgs args, ConvGeom cg) {
  extern __shared__ __attribute__((aligned(16))) char cxf[];
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
  const int task = xcd_task(blockIdx.x, gridDim.x);
  int jx = 0;
  while (jx + 1 < args.njobs && task >= args.task_end[jx]) ++jx;
  const FactorJobDev& J = args.job[jx];
  const OpDev& op = J.x;
  const int split = task - J.task_begin;  // one unit: task = split
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t b0 = (int64_t)split * cg.B / J.splits, b1 = (int64_t)(split + 1) * cg.B / J.splits;
  const int gt = tid % XF_GROUP, grp = wave / XF_GW;
  const int nsp = (cg.xs_np + XF_GROUP - 1) / XF_GROUP;
  u32x2* rec = reinterpret_cast<u32x2*>(cxf + XF_REC);
  uint16_t* tbl = reinterpret_cast<uint16_t*>(cxf + XF_TBL);
  // once per task: zero both buffers; the copy-base table from the kernel argument
  // (constant-index reads: a lane-indexed read of the argument copies it to scratch)
  for (int e = tid; e < 2 * XF_BUF / 16; e += XF_THREADS) reinterpret_cast<u32x4*>(cxf)[e] = u32x4{0u, 0u, 0u, 0u};
  if (tid < XF_CB / 2) {
    // (read through the kernel-argument pointer: cg is the second argument, at its
    // alignment after FactorArgs)
    typedef const __attribute__((address_space(4))) char kchar;
    typedef const __attribute__((address_space(4))) int kint;
    kchar* ka = (kchar*)__builtin_amdgcn_kernarg_segment_ptr();
    constexpr size_t cgo = (sizeof(FactorArgs) + alignof(ConvGeom) - 1) / alignof(ConvGeom) * alignof(ConvGeom);
    reinterpret_cast<int*>(tbl)[tid] = ((kint*)(ka + cgo + offsetof(ConvGeom, xf_cb)))[tid];
  }
  // the build-slot records (c, r, col): col even in padded coordinates; elements col ..
  // col + 2 of padded row r of channel c, their pairs written to copy (c, kj) at
  // ow = col - kj (kj even) or col + 1 - kj (kj odd), 0 <= ow < Wo (Wo even: a pair is
  // wholly in or out).  x: source dword + 8 (bits 0-15), elements in the image (bits
  // 16-18); y: 2 (r Wo + col) (bits 0-15), c (16-23), kernel columns in range (24-31)
  const int wp2 = cg.xs_wp2, rowp = cg.xs_hp * wp2;
  if (tid < XF_GROUP)
    for (int i = 0; i < nsp; ++i) {
      const int e = tid + i * XF_GROUP;
      uint32_t x = 0, y = 0;
      if (e < cg.xs_np) {
        const int c = e / rowp, rem = e - c * rowp, r = rem / wp2, col = 2 * (rem - r * wp2);
        const int h = r - op.ph;
        uint32_t dm = 0, km = 0;
        for (int d = 0; d < 3; ++d) {
          const int w = col + d - op.pw;
          if (h >= 0 && h < op.H && w >= 0 && w < op.W) dm |= 1u << d;
        }
        for (int kj = 0; kj < op.kw; ++kj) {
          const int ow = col - kj + (kj & 1);
          if (ow >= 0 && ow < cg.Wo) km |= 1u << kj;
        }
        x = (uint32_t)(dm ? (c * op.H + h) * op.W + col - op.pw + 8 : 0) | dm << 16;
        y = (uint32_t)(2 * (r * cg.Wo + col)) | (uint32_t)c << 16 | km << 24;
      }
      rec[i * XF_GROUP + tid] = u32x2{x, y};
    }
  __syncthreads();
  if (cg.ones >= 0)
    for (int e = tid; e < 2 * cg.L; e += XF_THREADS) {
      const int bs = e / cg.L, p = e - bs * cg.L;
      *reinterpret_cast<uint16_t*>(cxf + bs * XF_BUF + cg.xf_one + 2 * p) = 0x3f80;
    }
  constexpr int OUT = 0x7ffffff0;
  const int irec = op.C * op.H * op.W * 4;  // bytes of one image
  float v0[XF_SP][3];
  auto fetch = [&](int64_t b, const u32x2 (&rc)[XF_SP]) __attribute__((always_inline)) {
    const int seg = (int)((uint32_t)b / (uint32_t)cg.bseg);
    const float* src = seg_base(J, args.segs, seg) + (b - (int64_t)seg * cg.bseg) * op.sB;
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(src), 0, irec, 0x00020000);
#pragma unroll
    for (int i = 0; i < XF_SP; ++i) {
      if (i >= nsp) break;
      const int s0 = (int)(rc[i].x & 0xffffu) * 4 - 32;
#pragma unroll
      for (int d = 0; d < 3; ++d)
        v0[i][d] = __uint_as_float(
            __builtin_amdgcn_raw_buffer_load_b32(rs, (rc[i].x >> (16 + d)) & 1u ? s0 + 4 * d : OUT, 0, 0));
    }
  };
  auto records = [&](u32x2 (&rc)[XF_SP]) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < XF_SP; ++i) rc[i] = i < nsp ? rec[i * XF_GROUP + gt] : u32x2{0u, 0u};
  };
  // out-of-range kernel columns write to a dummy row (one dword per lane) instead of a
  // branch per copy
  const int NV = cg.xf_nv, KW = op.kw;
  const int dummy = cg.xf_dummy + 4 * lane;
  auto build = [&](char* buf, const u32x2 (&rc)[XF_SP]) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < XF_SP; ++i) {
      if (i >= nsp) break;
      uint32_t p0[3], p1[3];
      split3(v0[i][0], v0[i][1], p0[0], p0[1], p0[2]);
      split3(v0[i][1], v0[i][2], p1[0], p1[1], p1[2]);
      const int q = (int)(rc[i].y & 0xffffu), c = (int)((rc[i].y >> 16) & 0xffu);
      const uint32_t km = rc[i].y >> 24;
      const u32x4* tb = reinterpret_cast<const u32x4*>(tbl + c * 2 * XF_KW);
      const u32x4 t0 = tb[0], t1 = tb[1];  // this channel's copy bases, [kj][v]
#pragma unroll
      for (int kj = 0; kj < XF_KW; ++kj) {
        if (kj >= KW) break;
        const uint32_t wv = kj < 4 ? t0[kj] : t1[kj - 4];
        const bool in = (km >> kj) & 1u;
        const int qk = q + 2 * ((kj & 1) - kj);
#pragma unroll
        for (int v = 0; v < 2; ++v) {
          if (v >= NV) break;
          const int base = (int)(v ? wv >> 16 : wv & 0xffffu);
          char* d = buf + (in ? base + qk : dummy);
#pragma unroll
          for (int r = 0; r < 3; ++r)
            *reinterpret_cast<uint32_t*>(d + r * XF_PART) = (kj & 1) ? p1[r] : p0[r];
        }
      }
    }
  };
  // this wave's fragment set F (<= 4 block rows of the factor: A of block (bi, bj) is
  // fragment bi, B fragment bj -- one matrix) and its blocks as pairs of F indices, from
  // a fixed menu of patterns (XF_PAT), so one k-step reads |F| fragments for up to 4
  // blocks (LeNet-5's conv2: 14 fragment reads per k-step for 15 blocks instead of 30;
  // at two 8-byte reads per fragment and part the LDS was the bound)
  const int gw = wave % XF_GW, m = lane & 31, hh = lane >> 5;
  auto row_off = [&](int f) __attribute__((always_inline)) {
    if (f < op.cols) {
      const int kk = op.kh * op.kw, c = f / kk, rr = f - c * kk, ki = rr / op.kw, kj = rr - ki * op.kw;
      const int v = (cg.xf_vmap >> (2 * ki)) & 3;
      return (int)tbl[c * 2 * XF_KW + 2 * kj + v] + 2 * ki * cg.Wo;
    }
    return f == cg.ones ? cg.xf_one : cg.xf_zero;
  };
  int wcode = 0;  // (constant-index reads of the argument: see mode 5)
#pragma unroll
  for (int t = 0; t < XF_GW; ++t) {
    int e = cg.xf_wave[t];
    asm volatile("" : "+s"(e));
    wcode = gw == t ? e : wcode;
  }
  const int pat = wcode & 15;  // bits 4 + 3 q .. : F[q]
  int offF[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) offF[q] = row_off(32 * ((wcode >> (4 + 3 * q)) & 7) + m) + 16 * hh;
  floatx16 acc[XF_BPW], acc2[XF_D2];
#pragma unroll
  for (int i = 0; i < XF_BPW; ++i)
#pragma unroll
    for (int v = 0; v < 16; ++v) acc[i][v] = 0.f;
#pragma unroll
  for (int i = 0; i < XF_D2; ++i)
#pragma unroll
    for (int v = 0; v < 16; ++v) acc2[i][v] = 0.f;
  // the last k-step's positions past L (L even): fragments masked by dword
  const int nks = cg.xf_nks, last = nks - 1;
  const int vc = min(max(cg.L - (16 * last + 8 * hh), 0), 8);
  uint32_t amask[4];
#pragma unroll
  for (int d = 0; d < 4; ++d) amask[d] = 2 * d + 1 < vc ? 0xffffffffu : 0u;
  auto rd8 = [&](const char* p) __attribute__((always_inline)) {  // 8 bf16 from two 8-byte reads
    const u32x2 lo = *reinterpret_cast<const u32x2*>(p), hi2 = *reinterpret_cast<const u32x2*>(p + 8);
    return __builtin_bit_cast(bf16x8, u32x4{lo.x, lo.y, hi2.x, hi2.y});
  };
  auto mask_all = [&](X3Frag* F, int nf) __attribute__((always_inline)) {  // (in place)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (q >= nf) break;
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        u32x4 w = __builtin_bit_cast(u32x4, F[q].p[r]);
#pragma unroll
        for (int d = 0; d < 4; ++d) w[d] &= amask[d];
        F[q].p[r] = __builtin_bit_cast(bf16x8, w);
      }
    }
  };
  // one register set: after the block that uses a fragment last in this k-step, the
  // fragment is reloaded for the next one, so each load has the following blocks'
  // MFMAs to land (two whole sets of 4 fragments left no registers for the rest:
  // spills).  The block orders of XF_PAT put a fragment's last use before the next
  // k-step's first use wherever the pattern allows.  The last k-step's fragments are
  // masked in place (a zero A or B element zeroes the product).
  auto mma_pat = [&](const char* buf, auto PI) __attribute__((always_inline)) {
    constexpr XfPat P = XF_PAT[decltype(PI)::value];
    constexpr int NF = xf_pat_frags(P);
    X3Frag F[NF];
    auto load = [&](int t, int q) __attribute__((always_inline)) {
#pragma unroll
      for (int r = 0; r < 3; ++r) F[q].p[r] = rd8(buf + r * XF_PART + offF[q] + 32 * t);
    };
    // (first reads in the loop's order -- by last use -- so the wait at the loop head
    // holds for the entry as for the back edge; in fragment order it was lgkmcnt(0);
    // the last k-step peeled: a mask at the loop head made every k-step wait for all
    // of its reads)
#pragma unroll
    for (int s2 = 0; s2 < P.n; ++s2)
#pragma unroll
      for (int q = 0; q < NF; ++q)
        if (xf_pat_last_use(P, q) == s2) load(0, q);
    auto prod = [&](int s2) __attribute__((always_inline)) {  // (s2: unrolled constant)
      if (P.a[s2] == P.b[s2]) x3_four(acc[s2], acc2[xf_pat_diag(P, s2)], F[P.a[s2]]);
      else x3_six(acc[s2], F[P.a[s2]], F[P.b[s2]]);
    };
    for (int t = 0; t < last; ++t) {
#pragma unroll
      for (int s2 = 0; s2 < P.n; ++s2) {
        prod(s2);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int q = 0; q < NF; ++q)
          if (xf_pat_last_use(P, q) == s2) load(t + 1, q);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    mask_all(F, NF);
#pragma unroll
    for (int s2 = 0; s2 < P.n; ++s2) prod(s2);
  };
  auto mma = [&](const char* buf) __attribute__((always_inline)) {
    switch (pat) {
      case 0: mma_pat(buf, std::integral_constant<int, 0>{}); break;
      case 1: mma_pat(buf, std::integral_constant<int, 1>{}); break;
      case 2: mma_pat(buf, std::integral_constant<int, 2>{}); break;
      case 3: mma_pat(buf, std::integral_constant<int, 3>{}); break;
      case 4: mma_pat(buf, std::integral_constant<int, 4>{}); break;
      case 5: mma_pat(buf, std::integral_constant<int, 5>{}); break;
      case 6: mma_pat(buf, std::integral_constant<int, 6>{}); break;
      default: break;
    }
  };
  // phases as mode 5: group i % 2 multiplies image i, the other builds image i + 1 and
  // loads image i + 3; one straight-line loop per group
  const int64_t nimg = b1 - b0;
  auto phase_mma = [&](int64_t i) __attribute__((always_inline)) {
    if (i < nimg) mma(cxf + (int)(i & 1) * XF_BUF);
    __syncthreads();
  };
  auto phase_build = [&](int64_t i) __attribute__((always_inline)) {
    if (i + 1 < nimg) {
      u32x2 rc[XF_SP];
      records(rc);
      build(cxf + (int)((i + 1) & 1) * XF_BUF, rc);
      if (i + 3 < nimg) fetch(b0 + i + 3, rc);
    }
    __syncthreads();
  };
  if (grp == 0) {
    if (nimg > 0) {
      u32x2 rc[XF_SP];
      records(rc);
      fetch(b0, rc);
      build(cxf, rc);
      if (nimg > 2) {
        fetch(b0 + 2, rc);
#pragma unroll
        for (int i = 0; i < XF_SP; ++i) asm volatile("" ::"v"(v0[i][0]), "v"(v0[i][1]), "v"(v0[i][2]));  // (landed)
      }
    }
    __syncthreads();
    for (int64_t i = 0; i < nimg; i += 2) {
      phase_mma(i);
      phase_build(i + 1);
    }
  } else {
    if (nimg > 1) {
      u32x2 rc[XF_SP];
      records(rc);
      fetch(b0 + 1, rc);
    }
    __syncthreads();
    for (int64_t i = 0; i < nimg; i += 2) {
      phase_build(i);
      phase_mma(i + 1);
    }
  }
  // group 1's partial sums added to group 0's (fixed order), then the diagonal blocks'
  // acc + acc2 + acc2^T (the transpose through a per-wave LDS tile: a wave's LDS
  // operations complete in order), stored by group 0 (its accumulator reads in flight
  // across the exchange)
  float* red = reinterpret_cast<float*>(cxf);
  constexpr int XF_SETS = XF_BPW + XF_D2;
  const int nblk = pat < XF_NPAT ? xf_pat_blocks(pat) : 0;
  auto at = [&](int i, int v) __attribute__((always_inline)) {
    const int bi = (wcode >> (4 + 3 * xf_pat_a(pat, i))) & 7, bj = (wcode >> (4 + 3 * xf_pat_b(pat, i))) & 7;
    const int ti = bi >> 1, tj = bj >> 1;
    float* o = J.slab + ((size_t)(ti * (ti + 1) / 2 + tj) * J.sstride + split) * TILE * TILE +
               (bi & 1) * 32 * TILE + (bj & 1) * 32;
    return &o[acc_row(v, lane) * TILE + (lane & 31)];
  };
  float old[XF_BPW][16];
  if (grp == 1) {
#pragma unroll
    for (int i = 0; i < XF_SETS; ++i)
#pragma unroll
      for (int v = 0; v < 16; ++v)
        red[((gw * XF_SETS + i) * 16 + v) * 64 + lane] = i < XF_BPW ? acc[i][v] : acc2[i - XF_BPW][v];
  } else {
    load_partials(J, nblk, old, at);
  }
  __syncthreads();
  if (grp == 1) return;
#pragma unroll
  for (int i = 0; i < XF_BPW; ++i)
#pragma unroll
    for (int v = 0; v < 16; ++v) acc[i][v] += red[((gw * XF_SETS + i) * 16 + v) * 64 + lane];
#pragma unroll
  for (int i = 0; i < XF_D2; ++i)
#pragma unroll
    for (int v = 0; v < 16; ++v) acc2[i][v] += red[((gw * XF_SETS + XF_BPW + i) * 16 + v) * 64 + lane];
  float* tr = red + XF_GW * XF_SETS * 16 * 64 + gw * 32 * 33;  // this wave's 32 x 33 tile
  int d = 0;
#pragma unroll
  for (int i = 0; i < XF_BPW; ++i) {
    if (i >= nblk) break;
    if (xf_pat_a(pat, i) != xf_pat_b(pat, i)) continue;
    floatx16 y = acc2[0];
#pragma unroll
    for (int v = 0; v < 16; ++v) y[v] = d ? acc2[1][v] : y[v];
#pragma unroll
    for (int v = 0; v < 16; ++v) tr[acc_row(v, lane) * 33 + (lane & 31)] = y[v];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int v = 0; v < 16; ++v) acc[i][v] += y[v] + tr[(lane & 31) * 33 + acc_row(v, lane)];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // (the tile's reads before its next writes)
    ++d;
  }
  put_partials(J, nblk, acc, old, at);
}

// Channel-major factors with n <= 8 (the G of a conv layer with few output
// channels, e.g. LeNet-5's conv1: 6): F = sum over (image, position) of g g^T is
// n(n+1)/2 FMAs per position against n loads -- an HBM stream, not MFMA work.  Each
// thread takes runs of 4 positions of the task's images (float4 loads, coalesced
// along positions, no LDS staging), keeps the lower triangle in registers, and the
// workgroup sums it in a fixed order (wave shuffles, then the 4 waves) into the
// same 16x16 slab / accumulator block the MFMA kernel writes.  (n = 9..16 stays on
// the MFMA kernel: 136 partial sums per thread cost more to reduce than they save.)
template <int NMAX>
__global__ __launch_bounds__(NTHREADS) void kfac_factor_channel_small(FactorArgs args, ConvGeom cg) {
  constexpr int NT = NMAX * (NMAX + 1) / 2;
  __shared__ float part[NTHREADS / 64][NT];
  const int task = xcd_task(blockIdx.x, gridDim.x);
  int jx = 0;
  while (jx + 1 < args.njobs && task >= args.task_end[jx]) ++jx;
  const FactorJobDev& J = args.job[jx];
  const OpDev& op = J.x;
  const int split = task - J.task_begin;  // one unit: task = split
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n = op.cols;
  const int64_t b0 = (int64_t)split * cg.B / J.splits, b1 = (int64_t)(split + 1) * cg.B / J.splits;
  // (image, 4-position run) pairs of the task: 32-bit index math (a task's pairs and a
  // job's images fit 32 bits; the 64-bit divisions cost as much issue as the FMAs)
  const uint32_t L4 = (uint32_t)(op.L >> 2), per = (uint32_t)(b1 - b0) * L4;
  float acc[NT];
#pragma unroll
  for (int e = 0; e < NT; ++e) acc[e] = 0.f;
  // PP (image, run) pairs per trip, their PP x n float4 loads issued together
  constexpr int PP = 2;
  auto src_of = [&](uint32_t q) {
    const uint32_t img = q / L4, r4 = q - img * L4;
    // image b0 + img of the job: batch seg of the queued batches, image bi in it
    const uint32_t ab = (uint32_t)b0 + img, seg = ab / (uint32_t)cg.bseg;
    return seg_base(J, args.segs, (int)seg) + (int64_t)(ab - seg * cg.bseg) * op.sB + 4 * r4;
  };
  for (uint32_t q = tid; q < per; q += PP * NTHREADS) {
    const float* sp[PP];
    bool ok[PP];
#pragma unroll
    for (int h = 0; h < PP; ++h) {
      ok[h] = h == 0 || q + h * NTHREADS < per;
      sp[h] = ok[h] ? src_of(q + h * NTHREADS) : sp[0];
    }
    floatx4 x[PP][NMAX];
#pragma unroll
    for (int c = 0; c < NMAX; ++c)
#pragma unroll
      for (int h = 0; h < PP; ++h) {
        const bool in = c < n;  // (channels past n: zero rows of the triangle)
        x[h][c] = in ? *reinterpret_cast<const floatx4*>(sp[h] + c * op.L) : floatx4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
    for (int h = 1; h < PP; ++h)
      if (!ok[h]) {
#pragma unroll
        for (int c = 0; c < NMAX; ++c) x[h][c] = floatx4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
    for (int h = 0; h < PP; ++h)
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int i = 0, e = 0; i < NMAX; ++i)
#pragma unroll
          for (int j = 0; j <= i; ++j, ++e) acc[e] = fmaf(x[h][i][u], x[h][j][u], acc[e]);
  }
#pragma unroll
  for (int e = 0; e < NT; ++e) {
    float v = acc[e];
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    if (lane == 0) part[wave][e] = v;
  }
  __syncthreads();
  float* out = J.slab + (size_t)split * TILE * TILE;  // block 0 of tile 0
  for (int e = tid; e < NT; e += NTHREADS) {
    int i = 0;
    while ((i + 1) * (i + 2) / 2 <= e) ++i;
    const int j = e - i * (i + 1) / 2;
    const float t = (part[0][e] + part[1][e]) + (part[2][e] + part[3][e]);
    float* at1 = &out[i * TILE + j];
    float* at2 = &out[j * TILE + i];
    if (!J.accum) {
      *at1 = t;
      *at2 = t;
    } else {
      const float v = J.sbeta == 0.f ? J.alpha * t : fmaf(J.sbeta, *at1, J.alpha * t);
      *at1 = v;
      *at2 = v;
    }
  }
}

// Channel-major factors with 8 < n <= 32 (LeNet-5's conv2 G: 16 channels x 100
// positions per image) in bf16x3, fragments straight from HBM: a channel's positions
// are contiguous, so a lane's fragment -- 8 consecutive positions of one channel -- is
// two float4 loads, split in registers (x3_split8); one 32 x 32 diagonal block, four
// MFMAs per 16 positions (x3_four).  Each wave takes whole images (images w, w + 4, ..
// of the task), its k-steps flattened over them with XC_D k-steps of loads in flight;
// the 4 waves' sums meet in LDS in wave order, then acc + acc2 + acc2^T.  (It replaces
// the LDS-staged fp32 kernel there: an HBM stream at 2.2 TB/s.)
constexpr int XC_D = 4;  // k-steps of loads in flight per wave
__global__ __launch_bounds__(NTHREADS) void kfac_factor_channel_x3(FactorArgs args, ConvGeom cg) {
  __shared__ float red[2 * (NTHREADS / 64 - 1)][16][64];
  __shared__ float tr[32][33];
  const int task = xcd_task(blockIdx.x, gridDim.x);
  int jx = 0;
  while (jx + 1 < args.njobs && task >= args.task_end[jx]) ++jx;
  const FactorJobDev& J = args.job[jx];
  const OpDev& op = J.x;
  const int split = task - J.task_begin;  // one unit: task = split
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n = op.cols, L = (int)op.L, m = lane & 31, hh = lane >> 5;
  const int64_t b0 = (int64_t)split * cg.B / J.splits, b1 = (int64_t)(split + 1) * cg.B / J.splits;
  const int nks = (L + 15) / 16;
  const int nimg = b1 - b0 > wave ? (int)((b1 - b0 - wave + 3) / 4) : 0;
  const int total = nimg * nks;  // this wave's k-steps
  // cursor of the next k-step to load: image j of the wave, k-step t; its channel row
  const float* rowp = nullptr;
  int j = 0, t = 0;
  auto image_row = [&](int jj) __attribute__((always_inline)) {
    const uint32_t ab = (uint32_t)(b0 + wave + 4 * (int64_t)jj), seg = ab / (uint32_t)cg.bseg;
    return seg_base(J, args.segs, (int)seg) + (int64_t)(ab - seg * cg.bseg) * op.sB + (int64_t)min(m, n - 1) * L;
  };
  if (total > 0) rowp = image_row(0);
  auto load = [&](float (&x)[8]) __attribute__((always_inline)) {
    const int p = 16 * t + 8 * hh;
    const bool r0 = m < n && p < L, r1 = m < n && p + 4 < L;
    const floatx4 lo = r0 ? *reinterpret_cast<const floatx4*>(rowp + p) : floatx4{0.f, 0.f, 0.f, 0.f};
    const floatx4 hi = r1 ? *reinterpret_cast<const floatx4*>(rowp + p + 4) : floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      x[e] = lo[e];
      x[4 + e] = hi[e];
    }
    if (++t == nks) {
      t = 0;
      if (++j < nimg) rowp = image_row(j);
      else j = nimg;
    }
  };
  floatx16 acc, acc2;
#pragma unroll
  for (int v = 0; v < 16; ++v) acc[v] = acc2[v] = 0.f;
  // ring of XC_D k-steps: step s multiplies slot s % XC_D, then reloads it for s + XC_D
  // (unconditionally: past the wave's last k-step the cursor re-reads its last image,
  // unused -- a conditional load made every wait vmcnt(0))
  if (total > 0) {
    float x[XC_D][8];
#pragma unroll
    for (int d = 0; d < XC_D; ++d) load(x[d]);
    int s = 0;
    for (; s + XC_D <= total; s += XC_D) {
#pragma unroll
      for (int d = 0; d < XC_D; ++d) {
        const X3Frag f = x3_split8(x[d]);
        load(x[d]);
        x3_four(acc, acc2, f);
      }
    }
#pragma unroll
    for (int d = 0; d < XC_D; ++d)
      if (s + d < total) x3_four(acc, acc2, x3_split8(x[d]));
  }
  // the 4 waves' sums in wave order (deterministic), then acc + acc2 + acc2^T
  if (wave > 0)
#pragma unroll
    for (int v = 0; v < 16; ++v) {
      red[2 * (wave - 1)][v][lane] = acc[v];
      red[2 * (wave - 1) + 1][v][lane] = acc2[v];
    }
  __syncthreads();
  if (wave > 0) return;
  for (int w = 0; w < NTHREADS / 64 - 1; ++w)
#pragma unroll
    for (int v = 0; v < 16; ++v) {
      acc[v] += red[2 * w][v][lane];
      acc2[v] += red[2 * w + 1][v][lane];
    }
#pragma unroll
  for (int v = 0; v < 16; ++v) tr[acc_row(v, lane)][m] = acc2[v];
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
  for (int v = 0; v < 16; ++v) acc[v] += acc2[v] + tr[m][acc_row(v, lane)];
  float* out = J.slab + (size_t)split * TILE * TILE;  // block (0, 0) of slab tile 0
  put_partial(J, acc, [&](int v) { return &out[acc_row(v, lane) * TILE + m]; });
}

// KFAC_CONV_SMALL=0: channel factors with n <= 8 on the MFMA kernel (A/B checks)
static bool conv_small_off() { return !knobs().conv_small; }
// the register-triangle kernel takes channel factors with n <= 8 (an n = 16 instance --
// 136 sums per thread, 256 VGPRs -- ran LeNet-5's conv2 G at 0.63 ms per pass against
// 0.17 on the MFMA kernel, `profiles/r06z10/`)
static bool channel_small(const ConvGeom& g) { return !conv_small_off() && g.n <= 8; }

// Geometry of a conv job on the LDS-staged kernel; false: the job takes the
// register-staged path (images too large, channel blocks not float4-shaped, or an
// empty batch).  A multi-batch job's images are its nseg batches' images in order.
// smallest factor on mode 4: n in 17..32 (one block, LeNet-5's conv1 A) measured slower
// here than on the fp32 kernel's three 16x16 blocks (313 vs 139 us per launch, the
// im2col build of 784 positions per image costs more than the MFMAs save; profiles/r06g/);
// those factors take mode 5 (column copies, no im2col) where its geometry fits
constexpr int CX3_MIN_N = 33;
// LDS of the mode-4 workgroup: at most 131 KB, so a 29 KB inversion workgroup of an
// overlapped invert() still fits on the CU (160 KB)
constexpr int CX3_LDS_MAX = 134144;

// Mode 4 (kfac_factor_conv_x3): an im2col operand with n > 32 whose padded image and
// im2col chunk fit the LDS; positions per chunk LPC as large as fits (one chunk per
// image when the whole image does).
static bool conv_x3_geom(const kfac_operand& o, ConvGeom& g) {
  const int n = g.n;
  if (n < CX3_MIN_N || (int64_t)o.C * o.H * o.W > CONV_SRC_MAX || o.sh <= 0 || o.sw <= 0) return false;
  g.nb = (int)cdiv(n, 32);
  g.nq = g.nb * (g.nb + 1) / 2;
  // (at most 3 blocks per wave, n <= 192: 4 need ~300 registers with the build's)
  if (g.nq > 3 * CX3_WAVES) return false;
  // one block (17 <= n <= 32: LeNet-5's conv1 A, n = 26 over 784 positions) or three:
  // its k-steps interleaved over 8 / 2 waves
  g.kw = g.nq == 1 ? CX3_WAVES : g.nq == 2 ? CX3_WAVES / 2 : g.nq <= 4 ? 2 : 1;
  g.Wp = o.W + 2 * o.pw;
  g.plane = (o.H + 2 * o.ph) * g.Wp;
  g.imgf = o.C * g.plane;
  g.L = (int)o.L;
  g.Wo = o.Wo;
  g.sh = o.sh;
  g.sw = o.sw;
  g.src = o.C * o.H * o.W;
  g.ones = o.has_ones ? o.cols : -1;
  for (int lpc = (int)cdiv(o.L, 16) * 16; lpc >= 16; lpc -= 16) {
    const int nch = (int)cdiv(o.L, lpc), pitch = lpc + 8;
    const int64_t bytes = (int64_t)3 * 32 * g.nb * pitch * 2 + (int64_t)4 * 3 * g.imgf +
                          (int64_t)4 * ((int64_t)nch * lpc + n);
    if (bytes <= CX3_LDS_MAX && lpc / 8 <= CX3_THREADS) {
      g.LPC = lpc;
      g.nch = nch;
      g.pitch = pitch;
      // (kw > 1: the epilogue's partial-sum exchange, 8 waves x 16 x 64 floats)
      g.ldsb = (int)std::max<int64_t>(bytes, g.kw > 1 ? CX3_WAVES * 16 * 64 * 4 : 0);
      g.mode = 4;
      g.units = 1;
      return true;
    }
  }
  return false;
}

// Mode 5 (kfac_factor_conv_x3s): an im2col operand with 17 <= n <= 32 whose column
// copies fit XS_LDS_MAX and take at most XS_SP build slots per thread.  The
// copy row pitch and copy stride (multiples of 8 bf16) are searched for the fewest lanes
// of a 16-lane group on one 16-byte bank quad (their fragment reads differ by the copy
// and row offsets of xs_lane; the group offset is uniform), then the fewest bytes.
// the ds_read_b128 lane group (of lanes 0-31; 32-63 repeat it) of lane m:
// {0-3, 12-15, 20-27} and {4-11, 16-19, 28-31} (MI355X_MICROARCH.md, LDS)
static inline int b128_group(int m) { return (m >= 4 && m < 12) || (m >= 16 && m < 20) || m >= 28; }

static bool conv_x3s_geom(const kfac_operand& o, ConvGeom& g) {
  const int n = g.n;
  // (the build's pair slots: column stride 1, even Wo, kernel width <= XS_KW)
  if (n < 17 || n > 32 || o.sh <= 0 || o.sw != 1 || o.Ho <= 0 || o.Wo <= 0 || o.Wo % 2 != 0 ||
      o.kw > XS_KW)
    return false;
  const int hp = o.H + 2 * o.ph, g8 = (int)cdiv(o.Wo, 8), ncopy = o.C * o.kw;
  // (a wave's k-steps advance by whole output rows; every k-step two real groups)
  if (8 % g8 != 0 || o.Ho * g8 % 2 != 0) return false;
  const int wp2 = (o.W + 2 * o.pw + 1) / 2;
  const int64_t np = (int64_t)o.C * hp * wp2;
  if (np > (int64_t)XS_SP * XS_GROUP) return false;
  const int grp = o.Ho * g8, ones = o.has_ones ? o.cols : -1;
  // the data and bias rows' fragment offsets at row pitch pw, copy stride cs; their
  // 16-byte bank quads (a ds_read_b128 group of 16 lanes is conflict-free on 16
  // distinct quads); padding rows read the zero copy at any of 16 column offsets
  struct Item { int quad, lb, f; };
  auto items_of = [&](int64_t pw, int64_t cs, std::vector<Item>& it) {
    it.clear();
    for (int f = 0; f < o.cols + (ones >= 0 ? 1 : 0); ++f) {
      int k, row;
      xs_lane(f, o.cols, ones, o.kh, o.kw, ncopy, k, row);
      const int64_t lb = (k * cs + row * pw) * 2;
      it.push_back({(int)((lb / 16) % 16), (int)lb, f});
    }
  };
  int best_w = 1 << 30;
  int64_t best_b = 0;
  std::vector<Item> it;
  for (int pw = 8 * g8; pw < 8 * g8 + 128; pw += 8)
    for (int s = 0; s < 16; ++s) {
      int64_t cs = (int64_t)hp * pw;
      while ((cs / 8) % 16 != s) cs += 8;
      const int64_t bytes = (int64_t)2 * 3 * ((ncopy + 2) * cs * 2 + XS_ZPAD + XS_DUMMY);
      if (bytes > XS_LDS_MAX) continue;
      items_of(pw, cs, it);
      int cnt[16] = {0}, worst = 0;
      for (const Item& x : it) worst = std::max(worst, ++cnt[x.quad]);
      worst = (worst + 1) / 2;  // (split over the two lane groups)
      if (worst < best_w || (worst == best_w && bytes < best_b)) {
        best_w = worst;
        best_b = bytes;
        g.xs_pw = pw;
        g.xs_cs = (int)cs;
      }
    }
  if (best_w == 1 << 30) return false;
  // deal the rows to the two lane groups, each quad's users alternately, then pad each
  // group to 16 lanes with zero-copy reads on the quads it has least
  items_of(g.xs_pw, g.xs_cs, it);
  std::sort(it.begin(), it.end(), [](const Item& a, const Item& b) { return a.quad < b.quad; });
  std::vector<Item> grpl[2];
  int use[2][16] = {{0}};
  for (const Item& x : it) {
    int q = use[0][x.quad] < use[1][x.quad] ? 0 : use[1][x.quad] < use[0][x.quad] ? 1
            : grpl[0].size() <= grpl[1].size() ? 0 : 1;
    if (grpl[q].size() == 16) q = 1 - q;
    grpl[q].push_back(x);
    ++use[q][x.quad];
  }
  const int64_t zb = (int64_t)(ncopy + 1) * g.xs_cs * 2;
  int fpad = n;
  for (int q = 0; q < 2; ++q)
    while (grpl[q].size() < 16) {
      int quad = 0;
      for (int t = 1; t < 16; ++t)
        if (use[q][t] < use[q][quad]) quad = t;
      const int col = (int)(((quad - (zb / 16) % 16) % 16 + 16) % 16);
      grpl[q].push_back({quad, (int)(zb + 16 * col), fpad++});
      ++use[q][quad];
    }
  for (int m = 0, c[2] = {0, 0}; m < 32; ++m) {
    const int q = b128_group(m);
    const Item& x = grpl[q][c[q]++];
    g.xs_lb[m] = x.lb;
    g.xs_f[m] = (int8_t)x.f;
  }
  g.xs_ncopy = ncopy;
  g.xs_hp = hp;
  g.xs_g8 = g8;
  g.xs_grp = grp;
  g.xs_np = (int)np;
  g.xs_wp2 = wp2;
  g.L = (int)o.L;
  g.Wo = o.Wo;
  g.sh = o.sh;
  g.sw = o.sw;
  g.ones = ones;
  // (the epilogue's partial-sum exchange: 2 x 7 waves x 16 x 64 floats, a 32 x 33 transpose)
  g.ldsb = (int)std::max<int64_t>(best_b, 2 * (XS_WAVES - 1) * 16 * 64 * 4 + 32 * 33 * 4);
  g.nb = 1;
  g.nq = 1;
  g.mode = 5;
  g.units = 1;
  return true;
}

// Mode 6 (kfac_factor_conv_x3f): a stride-1 im2col operand with 32 < n <= 160 (<= 16
// blocks: 4 per multiplying wave), even Wo (bf16 pairs), kernel <= 8 x 8, C <= 16, whose
// copies fit in XF_PART and take at most XF_SP build slots per thread.
// Copy bases: the fragment row of feature (c, ki, kj) starts at 8-byte unit
// base(c, kj, v(ki)) + (ki Wo + shift) / 4; a 16-lane group of ds_read_b64 / ds_read2_b64
// is conflict-free when its 16 distinct units are distinct mod 16 (equal addresses
// broadcast: the zero rows).  A depth-first search over the copies' residues mod 16
// (in order of first use, <= 2^20 nodes) finds such bases (LeNet-5's conv2: 15 k nodes),
// then the copies are laid out in a chain that keeps the gaps between them small.
static bool xf_place(const kfac_operand& o, int nb, int nv, int vmap, const int* sft, int zo, int* res) {
  const int ncp = o.C * o.kw * nv, nc = ncp + 1;  // + the ones / zero region
  const int ones = o.has_ones ? o.cols : -1, ng = 2 * nb;
  auto feat = [&](int f, int& cp, int& off) {
    if (f < o.cols) {
      const int kk = o.kh * o.kw, c = f / kk, rr = f - c * kk, ki = rr / o.kw, kj = rr - ki * o.kw;
      const int v = (vmap >> (2 * ki)) & 3;
      cp = (c * o.kw + kj) * nv + v;
      off = (ki * o.Wo + sft[v]) / 4;
    } else {
      cp = ncp;
      off = f == ones ? 0 : zo;
    }
  };
  // uses[cp]: (group, offset) pairs, distinct
  std::vector<std::vector<std::pair<int, int>>> uses(nc);
  std::vector<int> first(nc, 1 << 30);
  for (int g = 0; g < ng; ++g)
    for (int f = 16 * g; f < 16 * g + 16; ++f) {
      int cp, off;
      feat(f, cp, off);
      bool dup = false;
      for (auto& u : uses[cp]) dup |= u.first == g && u.second == off;
      if (!dup) uses[cp].push_back({g, off});
      first[cp] = std::min(first[cp], g);
    }
  std::vector<int> order(nc);
  for (int i = 0; i < nc; ++i) order[i] = i;
  std::stable_sort(order.begin(), order.end(), [&](int x, int y) { return first[x] < first[y]; });
  std::vector<uint16_t> used(ng, 0);
  int64_t nodes = 0;
  std::function<bool(int)> dfs = [&](int k) -> bool {
    if (k == nc) return true;
    if (++nodes > (1 << 20)) return false;
    const int i = order[k];
    for (int r = 0; r < 16; ++r) {
      bool ok = true;
      for (auto& u : uses[i]) ok &= !((used[u.first] >> ((r + u.second) & 15)) & 1);
      if (!ok) continue;
      for (auto& u : uses[i]) used[u.first] |= (uint16_t)(1u << ((r + u.second) & 15));
      res[i] = r;
      if (dfs(k + 1)) return true;
      for (auto& u : uses[i]) used[u.first] &= (uint16_t)~(1u << ((r + u.second) & 15));
    }
    return false;
  };
  return dfs(0);
}

static bool conv_x3f_geom_new(const kfac_operand& o, ConvGeom& g);
// (the plan is made per call: the residue search and layout are memoized per shape --
// uncached they cost 7 ms per LeNet-5 pass)
static bool conv_x3f_geom(const kfac_operand& o, ConvGeom& g) {
  typedef std::array<int64_t, 12> Key;
  static std::mutex mu;
  static std::vector<std::pair<Key, std::pair<bool, ConvGeom>>> memo;
  const Key k{o.C, o.H, o.W, o.kh, o.kw, o.ph, o.pw, o.sh, o.sw, o.Ho * 65536 + o.Wo, o.cols * 2 + (o.has_ones ? 1 : 0),
              (int64_t)g.n};
  {
    std::lock_guard<std::mutex> lk(mu);
    for (auto& e : memo)
      if (e.first == k) {
        if (!e.second.first) return false;
        ConvGeom r = e.second.second;
        // (the fields set before this search: kept from the caller)
        r.B = g.B;
        r.bseg = g.bseg;
        g = r;
        return true;
      }
  }
  ConvGeom r = g;
  const bool ok = conv_x3f_geom_new(o, r);
  std::lock_guard<std::mutex> lk(mu);
  if (memo.size() < 64) memo.push_back({k, {ok, r}});
  if (ok) g = r;
  return ok;
}

static bool conv_x3f_geom_new(const kfac_operand& o, ConvGeom& g) {
  const int n = g.n;
  if (n <= 32 || o.sh != 1 || o.sw != 1 || o.Ho <= 0 || o.Wo <= 0 || o.Wo % 2 != 0 || o.kw > XF_KW ||
      o.kh > 8 || o.C > XF_CB / (2 * XF_KW) || (int64_t)o.C * o.H * o.W + 16 > 0xffff)
    return false;
  const int nb = (int)cdiv(n, 32), nq = nb * (nb + 1) / 2;
  if (nb != 4 && nb != 5) return false;  // (the fragment-sharing assignments, XF_PAT)
  const int hp = o.H + 2 * o.ph, wp2 = (o.W + 2 * o.pw + 1) / 2;
  const int64_t np = (int64_t)o.C * hp * wp2;
  if (np > (int64_t)XF_SP * XF_GROUP || 2 * (hp * o.Wo + 2 * wp2) > 0xffff) return false;
  // the shifts that align ki Wo + shift to 4 elements, one variant per distinct shift
  int nv = 0, vmap = 0, shifts[4];
  for (int ki = 0; ki < o.kh; ++ki) {
    const int sft = (4 - (ki * o.Wo) % 4) % 4;
    int v = 0;
    while (v < nv && shifts[v] != sft) ++v;
    if (v == nv) shifts[nv++] = sft;
    vmap |= v << (2 * ki);
  }
  if (nv > 2) return false;  // (the build writes two variants at most)
  const int ncp = o.C * o.kw * nv;
  const int nks = (int)cdiv(o.L, 16);
  const int cu = (hp * o.Wo + 3 + 3) / 4;  // 8-byte units per copy (elements shift .. shift + Hp Wo)
  const int zo = 4 * nks + 2;               // the zero copy after the ones copy (units)
  std::vector<int> res(ncp + 1);
  if (!xf_place(o, nb, nv, vmap, shifts, zo, res.data())) return false;
  // chain layout: the next copy is the one whose residue is reached with the least gap
  std::vector<std::vector<int>> pool(16);
  for (int i = ncp - 1; i >= 0; --i) pool[res[i]].push_back(i);
  std::vector<int> base(ncp + 1);
  int p = 0;
  for (int left = ncp; left > 0; --left)
    for (int gap = 0; gap < 16; ++gap) {
      auto& q = pool[(p + gap) & 15];
      if (q.empty()) continue;
      base[q.back()] = p + gap;
      q.pop_back();
      p += gap + cu;
      break;
    }
  while ((p & 15) != res[ncp]) ++p;
  base[ncp] = p;
  // ones copy, zero copy (16 nks + 8 bf16 of reads each), the dummy row (64 dwords, and
  // the last k-step's over-reads past any copy land before the part's end)
  const int dummy = 8 * (p + zo + 4 * nks + 4);
  if (dummy + 256 + 64 > XF_PART) return false;
  g.nb = nb;
  g.nq = nq;
  auto wave_code = [](int pat, std::initializer_list<int> f) {
    int c = pat, q = 0;
    for (int x : f) c |= x << (4 + 3 * q++);
    return c;
  };
  if (nb == 5) {
    g.xf_wave[0] = wave_code(0, {0, 1, 2, 3});
    g.xf_wave[1] = wave_code(1, {0, 1, 2, 4});
    g.xf_wave[2] = wave_code(2, {1, 2, 3, 4});
    g.xf_wave[3] = wave_code(3, {0, 2, 3, 4});
  } else {
    g.xf_wave[0] = wave_code(0, {0, 1, 2, 3});
    g.xf_wave[1] = wave_code(4, {0, 1, 2, 3});
    g.xf_wave[2] = wave_code(5, {0, 1, 2, 3});
    g.xf_wave[3] = wave_code(6, {0, 1, 2, 3});
  }
  g.xs_hp = hp;
  g.xs_wp2 = wp2;
  g.xs_np = (int)np;
  g.xf_nv = nv;
  g.xf_vmap = vmap;
  for (int c = 0; c < o.C; ++c)
    for (int kj = 0; kj < o.kw; ++kj)
      for (int v = 0; v < nv; ++v) {
        const int e = 16 * c + 2 * kj + v, b = 8 * base[(c * o.kw + kj) * nv + v] + 2 * shifts[v];
        g.xf_cb[e / 2] |= b << (16 * (e & 1));
      }
  g.xf_one = 8 * base[ncp];
  g.xf_zero = 8 * (base[ncp] + zo);
  g.xf_dummy = dummy;
  g.L = (int)o.L;
  g.xf_nks = nks;
  g.Wo = o.Wo;
  g.sh = o.sh;
  g.sw = o.sw;
  g.ones = o.has_ones ? o.cols : -1;
  g.ldsb = XF_LDS;
  g.mode = 6;
  g.units = 1;
  return true;
}

static bool conv_geom(const kfac_factor_job& j, ConvGeom& g) {
  const kfac_operand& o = j.x;
  const int64_t nseg = j.nseg > 1 ? j.nseg : 1;
  if ((o.layout != KFAC_PATCH && o.layout != KFAC_CHANNEL) || o.rows <= 0 || o.L <= 0 ||
      o.rows % o.L != 0 || nseg * (o.rows / o.L) > (1 << 30))
    return false;
  // (a CHANNEL operand with a ones column -- legal, unused by the hooks -- takes the
  // unstaged kernel: the channel kernels have no ones row)
  if (o.layout == KFAC_CHANNEL && o.has_ones) return false;
  const int n = o.cols + (o.has_ones ? 1 : 0);
  g = ConvGeom{};
  g.n = n;
  g.ones = o.has_ones ? o.cols : -1;
  g.bseg = (int)(o.rows / o.L);
  g.B = (int)(nseg * g.bseg);
  if (o.layout == KFAC_PATCH && knobs().conv_x3 &&
      (conv_x3s_geom(o, g) || conv_x3f_geom(o, g) || conv_x3_geom(o, g)))
    return true;
constexpr int KFAC_CONV_NARROW32 = 3;  // n in 17..32: 3 = three 16x16 blocks, 1 = one 32x32 block (A/B)
  g.mode = n <= 16 ? 2 : (n <= 32 ? KFAC_CONV_NARROW32 : 0);
  g.KR = g.mode >= 2 ? 4 : 2;
  int64_t lds;
  // Bank-conflict-free operand reads: an MFMA's 32 lanes of one lane group read 32
  // consecutive factor columns, column (c, ki, kj) at c*plane + ki*Wp + kj (PATCH) or
  // c*plane (CHANNEL) plus a lane-uniform offset.  ds_read_b32 banks are
  // (addr / 4) mod 32, so with Wp = kw and plane = kh*kw (PATCH) or plane = 1
  // (CHANNEL) modulo 32 every lane hits the bank of its own column index.  (16x16x4
  // CHANNEL blocks put two k-lanes in a group: their segments are 16 apart mod 32.)
  auto pad_to = [](int64_t v, int64_t r) { return v + (((r - v) % 32) + 32) % 32; };
  if (o.layout == KFAC_PATCH) {
    if ((int64_t)o.C * o.H * o.W > CONV_SRC_MAX) return false;
    g.Wp = o.W + 2 * o.pw;
    g.plane = (o.H + 2 * o.ph) * g.Wp;
    if (g.mode != 2) {  // (mode 3 too: its 16-lane groups read 16 consecutive columns)
      const int64_t Wp = pad_to(g.Wp, o.kw);
      const int64_t plane = pad_to((int64_t)(o.H + 2 * o.ph) * Wp, (int64_t)o.kh * o.kw);
      const int64_t need = o.C * plane + 2 * (int64_t)o.Ho * o.sh * Wp;
      if (need <= CONV_LDS_MAX) {
        g.Wp = (int)Wp;
        g.plane = (int)plane;
      }
    }
    g.Ho = o.Ho;
    g.rowstep = o.sh * g.Wp;
    g.T = o.Wo;
    g.G = (int)cdiv(o.Ho, g.KR);
    g.stride = o.sw;
    g.ones_base = o.C * g.plane;  // (= n - 1 mod 32: the bias column's own bank)
    // the padding columns of the last block all read the zero plane (one broadcast
    // address): put it on bank n mod 32, which no data column of that block uses
    // (at its unpadded place it shared a bank with one: 2-way conflicts)
    g.zero_base = g.ones_base + o.Ho * g.rowstep;
    g.zero_base += (int)((((int64_t)n - g.zero_base) % 32 + 32) % 32);
    lds = (int64_t)g.zero_base + o.Ho * g.rowstep;
    g.src = o.C * o.H * o.W;
  } else {
    const int64_t img = (int64_t)o.cols * o.L;
    if (o.L % 4 != 0 || o.sB % 4 != 0 || reinterpret_cast<uintptr_t>(o.ptr) % 16 != 0 ||
        img / 4 > CONV_SRC_MAX)
      return false;
    // a multi-batch job's float4 image loads start at every batch base (seg_ptrs is
    // a host table): one misaligned base sends the job to the per-batch launches
    if (nseg > 1) {
      const float* const* bases = reinterpret_cast<const float* const*>(j.seg_ptrs);
      for (int64_t s = 0; s < nseg; ++s)
        if (reinterpret_cast<uintptr_t>(bases[s]) % 16 != 0) return false;
    }
    const int segs = g.mode ? 4 * g.KR : g.KR;  // narrow: the 4 waves' segments too
    int Q = (int)cdiv(o.L, segs);
    if (g.mode >= 2) Q = (int)pad_to(Q, 16);
    g.rowstep = Q;
    g.plane = (int)pad_to((int64_t)segs * Q, 1);
    g.T = Q;
    g.G = 1;
    g.stride = 1;
    g.Ho = 1;
    g.zero_base = g.ones_base = o.cols * g.plane;
    lds = (int64_t)g.zero_base + g.plane;
    g.src = (int)(img / 4);
  }
  lds = std::max<int64_t>(lds, 3 * 16 * 64);
  if (lds > CONV_LDS_MAX) return false;
  const int nb = (int)cdiv(n, 32);
  g.nq = nb * (nb + 1) / 2;
  g.units = g.mode ? 1 : (int)cdiv(g.nq, 4 * CONV_CB);
  g.lds = (int)lds;
  // mode 8 (kfac_factor_channel_x3): CHANNEL factors with 8 < n <= 32, bf16x3 from HBM
  if (o.layout == KFAC_CHANNEL && n > 8 && n <= 32 && knobs().conv_x3) {
    g.mode = 8;
    g.units = 1;
  }
  return true;
}

template <int BPW>
static bool launch_conv_x3(const FactorArgs& args, const ConvGeom& g, int tasks, hipStream_t stream) {
  static const bool attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&kfac_factor_conv_x3<BPW>),
                                               hipFuncAttributeMaxDynamicSharedMemorySize,
                                               CX3_LDS_MAX) == hipSuccess;
  if (!attr) return false;
  hipLaunchKernelGGL(kfac_factor_conv_x3<BPW>, dim3(tasks), dim3(CX3_THREADS), (size_t)g.ldsb, stream, args, g);
  return true;
}

template <int LAYOUT>
static void launch_conv(const FactorArgs& args, const ConvGeom& g, int tasks, hipStream_t stream) {
  if (g.mode == 6) {
    static const bool attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&kfac_factor_conv_x3f),
                                                 hipFuncAttributeMaxDynamicSharedMemorySize,
                                                 XF_LDS) == hipSuccess;
    (void)attr;  // (a failed attribute surfaces as the launch error)
    hipLaunchKernelGGL(kfac_factor_conv_x3f, dim3(tasks), dim3(XF_THREADS), (size_t)g.ldsb, stream, args, g);
    return;
  }
  if (g.mode == 5) {
    static const bool attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&kfac_factor_conv_x3s),
                                                 hipFuncAttributeMaxDynamicSharedMemorySize,
                                                 XS_LDS_MAX) == hipSuccess;
    (void)attr;  // (a failed attribute surfaces as the launch error)
    hipLaunchKernelGGL(kfac_factor_conv_x3s, dim3(tasks), dim3(XS_THREADS), (size_t)g.ldsb, stream, args, g);
    return;
  }
  if (g.mode == 4) {
    const int bpw = (g.nq + CX3_WAVES - 1) / CX3_WAVES;
    const bool ok = bpw <= 1 ? launch_conv_x3<1>(args, g, tasks, stream)
                  : bpw == 2 ? launch_conv_x3<2>(args, g, tasks, stream)
                             : launch_conv_x3<3>(args, g, tasks, stream);
    (void)ok;  // (a failed attribute surfaces as the launch error below)
    return;
  }
  if (g.mode == 8) {
    hipLaunchKernelGGL(kfac_factor_channel_x3, dim3(tasks), dim3(NTHREADS), 0, stream, args, g);
    return;
  }
  if (LAYOUT == KFAC_CHANNEL && channel_small(g)) {
    // the exact channel count (LeNet-5 conv1: 6) sizes the register triangle and its
    // reduction; other counts take the next instance up (their extra rows are zero)
    if (g.n == 6)
      hipLaunchKernelGGL(kfac_factor_channel_small<6>, dim3(tasks), dim3(NTHREADS), 0, stream, args, g);
    else if (g.n <= 4)
      hipLaunchKernelGGL(kfac_factor_channel_small<4>, dim3(tasks), dim3(NTHREADS), 0, stream, args, g);
    else
      hipLaunchKernelGGL(kfac_factor_channel_small<8>, dim3(tasks), dim3(NTHREADS), 0, stream, args, g);
    return;
  }
  const size_t shmem = (size_t)g.lds * sizeof(float);
  const bool s1 = g.stride == 1;
  const int pm = (int)cdiv(g.src, NTHREADS);  // <= 8 by CONV_SRC_MAX
  // one instance per mode class, so each gets its own register budget: mode 0 (CB
  // blocks per wave), the one-block narrow modes 1 / 2 (CB = 1), mode 3
#define KFAC_CONV_LAUNCH(PM, S1, CBV, M3) \
  hipLaunchKernelGGL((kfac_factor_conv<LAYOUT, PM, S1, CBV, M3>), dim3(tasks), dim3(NTHREADS), shmem, stream, \
                     args, g)
#define KFAC_CONV_PICK(CBV, M3)                                                   \
  do {                                                                            \
    if (pm <= 4) {                                                                \
      if (s1) KFAC_CONV_LAUNCH(4, true, CBV, M3); else KFAC_CONV_LAUNCH(4, false, CBV, M3); \
    } else {                                                                      \
      if (s1) KFAC_CONV_LAUNCH(8, true, CBV, M3); else KFAC_CONV_LAUNCH(8, false, CBV, M3); \
    }                                                                             \
  } while (0)
  if (g.mode == 3)
    KFAC_CONV_PICK(CONV_CB, true);
  else if (g.mode != 0)
    KFAC_CONV_PICK(1, false);
  else
    KFAC_CONV_PICK(CONV_CB, false);
#undef KFAC_CONV_PICK
#undef KFAC_CONV_LAUNCH
}

// One block = one 4-row strip of one 64x64 tile.  Each float4 of the strip is
// summed by 4 threads over interleaved splits (part p: splits p, p+4, ...); the
// partials combine in LDS in part order (deterministic; no atomics), then
// F = beta*F + alpha*sum and the mirrored upper element (same value: F stays
// exactly symmetric).  16 blocks per tile keep jobs with one tile and many splits
// (narrow conv factors: ~1000 slabs) parallel.
constexpr int RSTRIP = 4;  // rows per reduce block

__global__ __launch_bounds__(NTHREADS) void kfac_factor_reduce(FactorArgs args) {
  __shared__ float4 part_sum[4][64];
  __shared__ float tot[RSTRIP][TILE + 1];
  // same proportional XCD mapping as the tiles launch: a tile's strips run on the XCD
  // whose L2 holds its freshly written slabs
  const int rb = xcd_task(blockIdx.x, gridDim.x);
  const int gtile = rb / (TILE / RSTRIP), s0 = (rb % (TILE / RSTRIP)) * RSTRIP;
  int j = 0;
  while (j + 1 < args.njobs && gtile >= args.tile_end[j]) ++j;
  const FactorJobDev& J = args.job[j];
  const int tile = gtile - J.tile_begin;
  int ti, tj;
  tri_decode(tile, ti, tj);
  const int i0 = ti * TILE, j0 = tj * TILE, n = J.n;
  const bool diag = ti == tj;
  const int part = threadIdx.x >> 6, f = threadIdx.x & 63;  // f: float4 of the 4 x 64 strip
  const int r = f >> 4, c4 = (f & 15) * 4;
  const float4* slab =
      reinterpret_cast<const float4*>(J.slab + (size_t)tile * J.sstride * TILE * TILE) +
      (((s0 + r) * TILE + c4) >> 2);
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  const int S = J.splits;
  int sp = part;
  for (; sp + 12 < S; sp += 16) {  // four splits of this part in flight
    const float4 a = slab[(size_t)(sp + 0) * (TILE * TILE / 4)];
    const float4 b = slab[(size_t)(sp + 4) * (TILE * TILE / 4)];
    const float4 c = slab[(size_t)(sp + 8) * (TILE * TILE / 4)];
    const float4 d = slab[(size_t)(sp + 12) * (TILE * TILE / 4)];
    acc.x += a.x; acc.y += a.y; acc.z += a.z; acc.w += a.w;
    acc.x += b.x; acc.y += b.y; acc.z += b.z; acc.w += b.w;
    acc.x += c.x; acc.y += c.y; acc.z += c.z; acc.w += c.w;
    acc.x += d.x; acc.y += d.y; acc.z += d.z; acc.w += d.w;
  }
  for (; sp < S; sp += 4) {
    const float4 a = slab[(size_t)sp * (TILE * TILE / 4)];
    acc.x += a.x; acc.y += a.y; acc.z += a.z; acc.w += a.w;
  }
  part_sum[part][f] = acc;
  __syncthreads();
  if (part == 0) {
    float4 t = part_sum[0][f];
#pragma unroll
    for (int p = 1; p < 4; ++p) {
      const float4 u = part_sum[p][f];
      t.x += u.x; t.y += u.y; t.z += u.z; t.w += u.w;
    }
    const float sum[4] = {t.x, t.y, t.z, t.w};
    const int gi = i0 + s0 + r;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int c = c4 + q, gj = j0 + c;
      float val = 0.f;
      if (gi < n && gj < n && !(diag && c > s0 + r)) {
        float* fp = J.F + (int64_t)gi * J.ldF + gj;
        val = J.beta == 0.f ? J.alpha * sum[q] : J.beta * (*fp) + J.alpha * sum[q];
        *fp = val;
      }
      tot[r][c] = val;
    }
  }
  __syncthreads();
  // mirror: F[j0 + c][i0 + s0 + rr] = tot[rr][c] (diag tiles: strictly-lower sources)
  const int c = threadIdx.x >> 2, rr = threadIdx.x & 3;
  const int si = i0 + s0 + rr, sj = j0 + c;
  if (si < n && sj < n && !(diag && c >= s0 + rr)) J.F[(int64_t)sj * J.ldF + si] = tot[rr][c];
}

// ------------------------------------------------------------------- host side
struct Plan {
  int tiles, splits;  // splits: slabs per tile (x3 thin jobs: splits - xsplits full K-splits)
  int xsplits;
  int units;  // workgroups per K-split: tiles, or a staged conv job's block groups
  int tasks;  // workgroups of the job
  int64_t chunk;
  size_t slab_bytes;
};

static int factor_n(const kfac_factor_job& j) { return j.x.cols + (j.x.has_ones ? 1 : 0); }

// K stages (BK rows each, never straddling two batches) of a job.
static int64_t job_sps(const kfac_factor_job& j) { return std::max<int64_t>(1, cdiv(j.x.rows, BK)); }
static int job_nseg(const kfac_factor_job& j) { return j.nseg > 1 ? j.nseg : 1; }
// a multi-batch job whose last batch is shorter (x.last_rows)
static bool job_ragged(const kfac_factor_job& j) {
  return j.nseg > 1 && j.x.last_rows > 0 && j.x.last_rows < j.x.rows;
}
static int64_t job_stages(const kfac_factor_job& j) {
  if (job_ragged(j)) return job_sps(j) * (j.nseg - 1) + std::max<int64_t>(1, cdiv(j.x.last_rows, BK));
  return job_sps(j) * job_nseg(j);
}
// K rows of a job (every batch; conv operands: images x positions) -- the profile's work
static int64_t job_krows(const kfac_factor_job& j) {
  if (job_ragged(j)) return j.x.rows * (j.nseg - 1) + j.x.last_rows;
  return j.x.rows * job_nseg(j);
}
// algorithmic bytes of a job's operand, read once: rows x cols x 4 (row-major, and the
// channel-major grads: images x positions x channels), the images themselves for the
// implicit im2col (images x C x H x W x 4)
static double job_operand_bytes(const kfac_factor_job& j) {
  const double rows = (double)job_krows(j);
  if (j.x.layout == KFAC_PATCH)
    return rows / (double)std::max<int64_t>(1, j.x.L) * (double)j.x.C * j.x.H * j.x.W * sizeof(float);
  return rows * j.x.cols * sizeof(float);
}

// Split K so that the grouped launch fills the chip's workgroup slots (256 CUs x 4
// resident workgroups) in as few dispatch rounds as possible with every task still
// running >= 8 stages (256 rows) of MFMA work.  One chunk length c (stages) is used
// for every job; tasks(c) = sum_j tiles_j * ceil(stages_j / c) falls with c, and the
// modelled time is (c + prologue/epilogue) * rounds: the smallest c that fits r
// rounds is found by bisection for r = 1..4 and the cheapest r wins.
// A job with a deferred-reduction accumulator keeps the accumulator's split count
// (its layout): its stage range is cut into that many equal chunks (trailing splits
// of a smaller batch may be empty and then contribute zero).
// Row-major operand with 16-byte-aligned rows: the LDS-DMA paths.
static bool job_glds(const kfac_factor_job& jb) {
  if (!(jb.x.layout == KFAC_ROWMAJOR && jb.x.rows > 0 && jb.x.cols >= 4 && (jb.x.cols % 4) == 0 &&
        (jb.x.ld % 4) == 0 && (reinterpret_cast<uintptr_t>(jb.x.ptr) % 16) == 0))
    return false;
  if (jb.nseg > 1 && jb.seg_ptrs) {  // (16-byte pieces start at every batch base)
    const uintptr_t* bases = reinterpret_cast<const uintptr_t*>(jb.seg_ptrs);
    for (int s = 0; s < jb.nseg; ++s)
      if (bases[s] % 16) return false;
  }
  return true;
}

// bf16x3 SYRK (kfac_factor_syrk3) for a row-major launch group: every job either
// LDS-eligible (16-byte rows, n > 32) or narrow (n <= 32, direct loads).
// Default: a group whose largest factor has n >= 2048 (measured A/B, same box: wide
// MLP 4097^2 factors 1.17e6 vs 9.4e5 img/s; the MNIST MLP's n <= 785 8.1e7 vs 1.0e8
// -- there the split pass's padded 6-byte images (785 -> 896, 129 -> 256 columns)
// cost as much as the fp32 kernel's whole launch).  KFAC_SYRK3=1 / 0 forces it.
static int syrk3_mode() { return knobs().syrk3; }

// bytes of a job's pre-split panel images (kfac_factor_syrk3; narrow jobs: none)

static bool syrk3_group(const kfac_factor_job* jobs, int njobs) {
  const int mode = syrk3_mode();
  if (mode == 0 || njobs <= 0) return false;
  int nmax = 0;
  for (int i = 0; i < njobs; ++i) {
    if (jobs[i].x.layout != KFAC_ROWMAJOR) return false;
    const int n = factor_n(jobs[i]);
    if (n > 32 && !job_glds(jobs[i])) return false;
    // (buffer loads: a batch's bytes are one 31-bit record range)
    if (n > 32 && jobs[i].x.rows * jobs[i].x.ld * (int64_t)sizeof(float) >= ((int64_t)1 << 31)) return false;
    nmax = std::max(nmax, n);
  }
  return nmax > 32 && (mode == 1 || nmax >= 2048);
}

// kfac_factor_tiles_x3 (fp32 panels, bf16x3 products split in registers) for every
// row-major group the split-pass kernel does not take (default; KFAC_TILES_X3=0: the
// fp32-MFMA kfac_factor_tiles).  MNIST MLP, same box, 2 reps: 1.21-1.23e8 vs
// 1.01e8 img/s, 81-82 vs 108 us per launch, the inversion beside the pass 0.41 vs
// 0.61 ms (2 SYRK waves per SIMD instead of 4).  Groups whose largest factor has
// n < 256 keep the fp32 kernel.  LeNet-5's fully connected factors (n <= 401) measured
// 1.34e7 vs 1.39e7 img/s with x3 in round 5; with round 6's conv kernels the pass is
// 2.01-2.02 vs 2.06 ms with x3 (0.26 vs 0.31 ms of fc factors, 3 reps alternating,
// `profiles/r06z13/`), so the threshold moved from 512 to 256.
static int tiles_x3_mode() { return knobs().tiles_x3; }

static bool tiles_x3_group(const kfac_factor_job* jobs, int njobs) {
  if (tiles_x3_mode() == 0 || njobs <= 0 || syrk3_group(jobs, njobs)) return false;
  int nmax = 0;
  for (int i = 0; i < njobs; ++i) {
    if (jobs[i].x.layout != KFAC_ROWMAJOR) return false;
    const int n = factor_n(jobs[i]);
    if (n > 32 && !job_glds(jobs[i])) return false;
    // (buffer loads: a batch's bytes are one 31-bit record range)
    if (n > 32 && jobs[i].x.rows * jobs[i].x.ld * (int64_t)sizeof(float) >= ((int64_t)1 << 31)) return false;
    nmax = std::max(nmax, n);
  }
  return nmax >= (tiles_x3_mode() == 1 ? 33 : 256);
}

static void plan_jobs(const kfac_factor_job* jobs, int njobs, Plan* plans,
                      int64_t slots = 0) {
  const bool s3 = syrk3_group(jobs, njobs);
  // resident workgroups per CU: 4 (32 KB of LDS each; kfac_factor_tiles_x3: 4 of two
  // waves -- 3 or 2 measured slower); kfac_factor_syrk3: S3D_WGS (49 KB each)
  if (slots <= 0) slots = (s3 ? S3D_WGS : 4) * 256;
  constexpr int64_t MIN_CHUNK = 8, OVERHEAD = 4;  // stages; ~per-task fixed cost in stages
  int64_t max_steps = 1;
  for (int i = 0; i < njobs; ++i) max_steps = std::max(max_steps, job_stages(jobs[i]));
  int64_t units[MAXJ];
  const bool x3 = !s3 && tiles_x3_group(jobs, njobs);
  for (int i = 0; i < njobs; ++i) {
    const int64_t t = cdiv(factor_n(jobs[i]), TILE);
    const int64_t t3 = cdiv(factor_n(jobs[i]), MT);
    ConvGeom cg;
    if (s3) units[i] = factor_n(jobs[i]) <= 32 ? 1 : t3 * (t3 + 1) / 2;
    else if (x3) units[i] = x3_units((int)factor_n(jobs[i]), (int)t);
    else units[i] = conv_geom(jobs[i], cg) ? cg.units : t * (t + 1) / 2;
  }
  // x3 jobs with thin-row pairs: the pair units are the slowest (30 MFMAs on 3
  // fragments per 16 rows: 1,606 vs 1,434 ns per stage for a full tile, profiles/r04am/),
  // so they take f/k more K-splits (x3_xsplits) and end with the full tiles
  auto xs_of = [&](int i, int64_t S) {
    const int t = (int)cdiv(factor_n(jobs[i]), TILE);
    return x3 && x3_thin(factor_n(jobs[i]), t) ? x3_xsplits(S) : 0;
  };
  // workgroups of job i at `splits` slabs per tile
  auto job_tasks = [&](int i, int64_t splits) {
    const int64_t xs = xs_of(i, splits);
    const int t = (int)cdiv(factor_n(jobs[i]), TILE);
    return units[i] * (splits - xs) + (int64_t)(t - 1) * xs * (xs > 0);
  };
  // (kfac_factor_tiles_x3: narrow jobs (n <= 32) at 4x the chunk's K-splits measured ~1 %
  // slower on the MLP line, profiles/r04ah/)
  auto job_splits = [&](int i, int64_t c) {
    const int64_t st = job_stages(jobs[i]);
    const int64_t sp = cdiv(st, c);
    const int t = (int)cdiv(factor_n(jobs[i]), TILE);
    if (x3 && x3_thin(factor_n(jobs[i]), t) && x3_pair_xs()) return std::min(st, sp + sp / x3_pair_xs());
    return sp;
  };
  auto tasks_at = [&](int64_t c) {
    int64_t n = 0;
    for (int i = 0; i < njobs; ++i)
      n += job_tasks(i, job_splits(i, c));
    return n;
  };
  int64_t best_c = std::max(MIN_CHUNK, max_steps), best_cost = -1;
  // (kfac_factor_tiles_x3 groups with thin-row pairs: one round -- MNIST MLP, same box:
  // 163.4 vs 170.3 / 167.4 us per launch at the two rounds the cost model picks; other
  // x3 groups keep the cost model's choice, which nothing measured against)
  bool any_thin = false;
  for (int i = 0; i < njobs && x3; ++i) any_thin |= x3_thin(factor_n(jobs[i]), (int)cdiv(factor_n(jobs[i]), TILE));
  // (kfac_factor_syrk3 groups, 2 workgroups per CU: up to 16 rounds, so a launch of
  // ~2,200 macro tiles (wide C5) can take 2 K-splits at 9 rounds instead of 1 at 4.3:
  // 1.61 vs 1.71 ms per launch, profiles/r05ac/)
  const int64_t max_rounds = any_thin ? 1 : (s3 ? 16 : 4);
  for (int64_t r = 1; r <= max_rounds; ++r) {
    int64_t lo = MIN_CHUNK, hi = std::max(MIN_CHUNK, max_steps);
    if (tasks_at(hi) > r * slots) continue;  // even one split per tile needs more rounds
    while (lo < hi) {
      const int64_t mid = (lo + hi) / 2;
      if (tasks_at(mid) <= r * slots) hi = mid; else lo = mid + 1;
    }
    const int64_t cost = (lo + OVERHEAD) * r;
    if (best_cost < 0 || cost < best_cost) { best_cost = cost; best_c = lo; }
  }
  for (int i = 0; i < njobs; ++i) {
    const int t = (int)cdiv(factor_n(jobs[i]), TILE);
    Plan& p = plans[i];
    p.tiles = t * (t + 1) / 2;
    p.units = (int)units[i];
    const int64_t steps = job_stages(jobs[i]);
    if (jobs[i].acc) {
      p.splits = jobs[i].acc_splits;
      p.xsplits = (int)xs_of(i, p.splits);
      p.chunk = cdiv(steps, (int64_t)(p.splits - p.xsplits));
      p.slab_bytes = 0;  // partials go to the caller's accumulator
      p.tasks = (int)job_tasks(i, p.splits);
      continue;
    }
    p.splits = (int)job_splits(i, best_c);
    ConvGeom cg;
    if (conv_geom(jobs[i], cg)) {
      // Tasks own whole images, the SAME number k each, and fill the resident slots
      // once: k = the fewest images per task that keep units x ceil(B / k) tasks
      // within the slots.  A workgroup's time is k times a per-image cost, so a mix of
      // 2- and 3-image tasks waited on the 3-image ones, and a CU running more
      // workgroups than another finished later (LeNet-5, batch 1024: conv2 A 68 us at
      // 400 splits -> 53 us at k = 2 (1,024 tasks); conv1 A 34 -> 27 us at k = 1;
      // `git show e37cdaa^:tools/microbench/conv_ab.hip`, KFAC_CONV_K overrides k)
      // (the n <= 8 channel kernel: half the slots -- its per-task reduction is the
      // larger cost there: conv1 G 15.7 / 12.4 / 13.2 us at k = 1 / 2 / 4)
      const bool small = jobs[i].x.layout == KFAC_CHANNEL && channel_small(cg);
      // (mode-0 instances are compiled for KFAC_CONV_OCC resident workgroups per CU;
      // modes 4-6 run one 512-thread workgroup per CU, mode 8 four of 256)
      const int64_t cslots = cg.mode == 0 ? (int64_t)KFAC_CONV_OCC * 256 : (cg.mode >= 4 && cg.mode <= 6) ? 256 : slots;
      // (a multi-batch launch -- thousands of images -- amortizes that reduction: the n <= 8
      // kernel then takes 4 workgroups per CU, twice the loads in flight of 2)
      const bool halve = small && cg.B <= 8 * cslots;
      int k = (int)std::max<int64_t>(1, cdiv((int64_t)cg.units * cg.B, halve ? cslots / 2 : cslots));
      if (knobs().conv_k > 0) k = knobs().conv_k;
      k = std::min(k, cg.B);
      p.splits = (int)cdiv(cg.B, k);
    }
    p.xsplits = (int)xs_of(i, p.splits);
    p.chunk = cdiv(steps, (int64_t)(p.splits - p.xsplits));
    p.slab_bytes = align_up((size_t)p.tiles * p.splits * TILE * TILE * sizeof(float), 256);
    p.tasks = (int)job_tasks(i, p.splits);
  }
}

static size_t accum_bytes(int n, int splits) {
  const int64_t t = cdiv(n, TILE);
  return align_up((size_t)(t * (t + 1) / 2) * splits * TILE * TILE * sizeof(float), 256);
}

static bool valid_operand(const kfac_operand& o) {
  if (o.cols < 0 || o.rows < 0 || (!o.ptr && o.rows > 0)) return false;
  switch (o.layout) {
    case KFAC_ROWMAJOR: return o.ld >= o.cols;
    case KFAC_CHANNEL: return o.L > 0 && o.sB >= 0;
    case KFAC_PATCH:
      return o.L > 0 && o.C > 0 && o.H > 0 && o.W > 0 && o.kh > 0 && o.kw > 0 && o.sh > 0 &&
             o.sw > 0 && o.ph >= 0 && o.pw >= 0 && o.Ho > 0 && o.Wo > 0 &&
             (int64_t)o.Ho * o.Wo == o.L && o.cols == o.C * o.kh * o.kw && o.kh < 65536 &&
             o.kw < 65536;
    default: return false;
  }
}

static void fill_dev(FactorJobDev& d, const kfac_factor_job& jb) {
  d.x = to_dev(jb.x);
  d.alpha = jb.alpha;
  d.beta = jb.beta;
  d.F = jb.F;
  d.ldF = jb.ldF;
  d.n = factor_n(jb);
  d.t = (int)cdiv(d.n, TILE);
  d.accum = jb.acc != nullptr;
  d.sbeta = jb.acc_beta;
  d.seg_off = -1;  // factor_group() places multi-batch bases
  d.nseg = job_nseg(jb);
  d.sps = (int)job_sps(jb);
  d.nst = job_stages(jb);
  d.rstage = -1;
  d.rw = d.rinv = 1.f;
  d.rdelta = 0;
  if (job_ragged(jb)) {
    d.rdelta = (int)(jb.x.rows - jb.x.last_rows);
    d.rstage = (int64_t)d.sps * (jb.nseg - 1);
    d.rw = (float)((double)jb.x.rows / (double)jb.x.last_rows);
    d.rinv = (float)((double)jb.x.last_rows / (double)jb.x.rows);
  }
}

// One reduce launch over `njobs` jobs whose slabs are described by d.slab/d.splits.
static void launch_reduce(FactorArgs& r, int tiles, hipStream_t stream) {
  if (tiles == 0) return;
  ProfScope ps(KFAC_PROF_FACTOR_REDUCE, stream);
  hipLaunchKernelGGL(kfac_factor_reduce, dim3(tiles * (TILE / RSTRIP)), dim3(NTHREADS), 0, stream,
                     r);
}

// The launch arguments of one grouped update: the tiles launch (`args`, `tasks`
// workgroups) and the reduce of the jobs without an accumulator (`red`, `rtiles`
// tiles).  Returns KFAC_EWORKSPACE when the slabs do not fit.
struct GroupLaunch {
  FactorArgs args, red;
  int tasks, rtiles;
};

static int prepare_group(const kfac_factor_job* jobs_in, int njobs, char* ws, size_t ws_bytes,
                         GroupLaunch& g) {
  const kfac_factor_job* jobs = jobs_in;
  Plan plans[MAXJ];
  plan_jobs(jobs, njobs, plans);
  FactorArgs& args = g.args;
  FactorArgs& red = g.red;  // the reduce launch: jobs reduced now (no accumulator)
  args = FactorArgs{};
  red = FactorArgs{};
  args.njobs = njobs;
  // split-major task order (each XCD a contiguous range of K-splits of all tiles):
  // 55 k vs 194 k KiB fetched per launch tile-major at equal time
  args.split_major = 1;
  int tasks = 0, rtiles = 0, nsegs = 0;
  size_t off = 0;
  for (int i = 0; i < njobs; ++i) {
    const kfac_factor_job& jb = jobs[i];
    FactorJobDev& d = args.job[i];
    fill_dev(d, jb);
    d.glds = job_glds(jb);
    d.x3pair = tiles_x3_group(jobs, njobs) && x3_thin(d.n, d.t);
    d.splits = plans[i].splits;
    d.xsplits = plans[i].xsplits;
    d.sstride = jb.acc && jb.acc_stride > 0 ? jb.acc_stride : d.splits;
    d.chunk = plans[i].chunk;
    if (d.nseg > 1) {  // kfac_factor_update keeps a launch within KSEG batch bases
      const float* const* bases = reinterpret_cast<const float* const*>(jb.seg_ptrs);
      d.seg_off = nsegs;
      for (int s = 0; s < d.nseg; ++s) args.segs[nsegs++] = bases[s];
    }
    if (jb.acc) {
      d.slab = jb.acc;
    } else {
      d.slab = reinterpret_cast<float*>(ws + off);
      off += plans[i].slab_bytes;
      FactorJobDev& e = red.job[red.njobs];
      e = d;
      e.tile_begin = rtiles;
      rtiles += plans[i].tiles;
      red.tile_end[red.njobs++] = rtiles;
    }
    d.task_begin = tasks;
    tasks += plans[i].tasks;
    args.task_end[i] = tasks;
  }
  g.tasks = tasks;
  g.rtiles = rtiles;
  return off > ws_bytes ? KFAC_EWORKSPACE : KFAC_OK;
}

static int factor_group(const kfac_factor_job* jobs, int njobs, char* ws, size_t ws_bytes,
                        hipStream_t stream) {
  GroupLaunch g;
  const int rc = prepare_group(jobs, njobs, ws, ws_bytes, g);
  if (rc != KFAC_OK) return rc;
  FactorArgs& args = g.args;
  FactorArgs& red = g.red;
  const int tasks = g.tasks, rtiles = g.rtiles;
  if (tasks == 0) return KFAC_OK;
  const bool s3 = syrk3_group(jobs, njobs);
  const bool x3 = tiles_x3_group(jobs, njobs);
  {
    // launch_groups() gives every channel-major / im2col job a group of its own
    // conv jobs whose images fit LDS: the image-staged kernel
    ConvGeom cg;
    const bool staged = njobs == 1 && conv_geom(jobs[0], cg);
    // one profile slot per kernel family (the name rocprofv3 reports), with the
    // launch's algorithmic flops: sum over jobs of K rows x n (n + 1)
    const int slot = s3 ? KFAC_PROF_FACTOR_SYRK3 : x3 ? KFAC_PROF_FACTOR_X3
                     : !staged ? KFAC_PROF_FACTOR_TILES
                     : (jobs[0].x.layout == KFAC_CHANNEL && channel_small(cg))
                         ? KFAC_PROF_FACTOR_CHANNEL_SMALL
                     : cg.mode == 8 ? KFAC_PROF_FACTOR_CHANNEL_X3
                     : cg.mode == 6 ? KFAC_PROF_FACTOR_CONV_X3F
                     : cg.mode == 5 ? KFAC_PROF_FACTOR_CONV_X3S
                     : cg.mode == 4 ? KFAC_PROF_FACTOR_CONV_X3 : KFAC_PROF_FACTOR_CONV;
    double work = 0.0, bytes = 0.0;
    if (prof_on())
      for (int i = 0; i < njobs; ++i) {
        work += (double)job_krows(jobs[i]) * factor_n(jobs[i]) * (factor_n(jobs[i]) + 1);
        bytes += job_operand_bytes(jobs[i]);
      }
    ProfScope ps(slot, stream, work, bytes);
    switch (jobs[0].x.layout) {
      case KFAC_CHANNEL:
        if (staged)
          launch_conv<KFAC_CHANNEL>(args, cg, tasks, stream);
        else
          hipLaunchKernelGGL(kfac_factor_tiles_channel, dim3(tasks), dim3(NTHREADS), 0, stream, args);
        break;
      case KFAC_PATCH:
        if (staged)
          launch_conv<KFAC_PATCH>(args, cg, tasks, stream);
        else
          hipLaunchKernelGGL(kfac_factor_tiles_patch, dim3(tasks), dim3(NTHREADS), 0, stream, args);
        break;
      default:
        {
          bool all_glds = true;
          for (int i = 0; i < njobs; ++i) all_glds &= args.job[i].glds != 0 || args.job[i].n <= 32;
          if (s3) {
            static const bool attr = hipFuncSetAttribute(
                reinterpret_cast<const void*>(&kfac_factor_syrk3),
                hipFuncAttributeMaxDynamicSharedMemorySize, S3D_LDS) == hipSuccess;
            if (!attr) return KFAC_ELAUNCH;
            hipLaunchKernelGGL(kfac_factor_syrk3, dim3(tasks), dim3(NTHREADS), S3D_LDS, stream, args);
          } else if (x3)
            hipLaunchKernelGGL(kfac_factor_tiles_x3, dim3(tasks), dim3(X3_THREADS), 0, stream, args);
          else if (all_glds)
            hipLaunchKernelGGL(kfac_factor_tiles_glds, dim3(tasks), dim3(NTHREADS), 0, stream, args);
          else
            hipLaunchKernelGGL(kfac_factor_tiles, dim3(tasks), dim3(NTHREADS), 0, stream, args);
        }
    }
    KFAC_CHECK_LAUNCH();
  }
  launch_reduce(red, rtiles, stream);
  KFAC_CHECK_LAUNCH();
  return KFAC_OK;
}

static size_t group_ws(const kfac_factor_job* jobs, int njobs) {
  Plan plans[MAXJ];
  plan_jobs(jobs, njobs, plans);
  size_t off = 0;
  for (int i = 0; i < njobs; ++i) off += plans[i].slab_bytes;
  return off;
}

}  // namespace kfac

using namespace kfac;

// Row-major jobs share launches (up to MAXJ each): their K-steps cost alike, so the
// planner's equal-step split balances them.  Each channel-major / im2col job gets
// a launch (and a plan) of its own: a K-step of a gather-bound operand costs far
// more than one of a row-major MFMA tile, and mixing them leaves the fast tasks
// idle behind the slow ones (LeNet-5: 1.35 ms grouped vs 0.94 ms per-job).
// `order` receives the caller's job index of each entry of `sorted`.
static void launch_groups(const kfac_factor_job* jobs, int njobs, std::vector<kfac_factor_job>& sorted,
                          std::vector<int>& order, std::vector<std::pair<int, int>>& groups) {
  sorted.clear();
  order.clear();
  groups.clear();
  for (int i = 0; i < njobs; ++i)
    if (jobs[i].x.layout == KFAC_ROWMAJOR) {
      sorted.push_back(jobs[i]);
      order.push_back(i);
    }
  const int nrm = (int)sorted.size();
  for (int g = 0; g < nrm; g += MAXJ) groups.emplace_back(g, std::min(MAXJ, nrm - g));
  for (int i = 0; i < njobs; ++i)
    if (jobs[i].x.layout != KFAC_ROWMAJOR) {
      groups.emplace_back((int)sorted.size(), 1);
      sorted.push_back(jobs[i]);
      order.push_back(i);
    }
}

extern "C" size_t kfac_factor_workspace_bytes(const kfac_factor_job* jobs, int njobs) {
  if (!jobs || njobs <= 0) return 0;
  std::vector<kfac_factor_job> sorted;
  std::vector<int> order;
  std::vector<std::pair<int, int>> groups;
  launch_groups(jobs, njobs, sorted, order, groups);
  size_t m = 0;
  for (const auto& g : groups) m = std::max(m, group_ws(sorted.data() + g.first, g.second));
  return m;
}

static int validate(const kfac_factor_job* jobs, int njobs) {
  if (njobs < 0 || (njobs > 0 && !jobs)) return KFAC_EINVAL;
  for (int i = 0; i < njobs; ++i) {
    const kfac_factor_job& j = jobs[i];
    if (!valid_operand(j.x) || !j.F || j.ldF < factor_n(j)) return KFAC_EINVAL;
    if ((int64_t)factor_n(j) > (int64_t)1 << 20) return KFAC_EINVAL;
    if (j.acc && (j.acc_splits <= 0 || j.acc_splits > (1 << 20))) return KFAC_EINVAL;
    if (j.acc && j.acc_stride != 0 && (j.acc_stride < j.acc_splits || j.acc_stride > (1 << 20)))
      return KFAC_EINVAL;
    if (j.nseg < 0 || (j.nseg > 1 && !j.seg_ptrs) || job_sps(j) > (1 << 30))
      return KFAC_EINVAL;
    if (j.x.last_rows < 0 || j.x.last_rows > j.x.rows ||
        (job_ragged(j) && j.x.layout != KFAC_ROWMAJOR))
      return KFAC_EINVAL;
  }
  return KFAC_OK;
}

extern "C" int kfac_factor_accum_plan(const kfac_factor_job* jobs, int njobs, int32_t* splits,
                                      size_t* bytes) {
  if (validate(jobs, njobs) != KFAC_OK || (njobs > 0 && (!splits || !bytes))) return KFAC_EINVAL;
  std::vector<kfac_factor_job> sorted;
  std::vector<int> order;
  std::vector<std::pair<int, int>> groups;
  launch_groups(jobs, njobs, sorted, order, groups);
  for (auto& j : sorted) j.acc = nullptr;  // plan as an immediate update of this batch
  for (const auto& g : groups) {
    Plan plans[MAXJ];
    plan_jobs(sorted.data() + g.first, g.second, plans);
    for (int k = 0; k < g.second; ++k) {
      const int i = order[g.first + k];
      splits[i] = plans[k].splits;
      bytes[i] = accum_bytes(factor_n(jobs[i]), plans[k].splits);
    }
  }
  return KFAC_OK;
}

// One launch group of kfac_factor_update.  A ragged multi-batch job (x.last_rows) runs
// in one launch on kfac_factor_tiles_x3 (and its narrow tasks); any other kernel, or a
// group past the launch's KSEG batch bases, takes it as two launches: the equal batches,
// then the last batch as a job of its own (alpha * rows / last_rows, adding).
static int update_group(const kfac_factor_job* gj, int n, void* workspace, size_t workspace_bytes,
                        kfac_stream_t stream) {
  bool ragged = false;
  int nbases = 0;
  for (int k = 0; k < n; ++k) {
    ragged |= job_ragged(gj[k]);
    nbases += job_nseg(gj[k]) > 1 ? gj[k].nseg : 0;
  }
  if (ragged && (!tiles_x3_group(gj, n) || nbases > KSEG)) {
    std::vector<kfac_factor_job> head(gj, gj + n), tail;
    for (kfac_factor_job& j : head) {
      if (!job_ragged(j)) continue;
      const float* const* bases = reinterpret_cast<const float* const*>(j.seg_ptrs);
      kfac_factor_job t = j;
      t.x.ptr = bases[j.nseg - 1];
      t.x.rows = j.x.last_rows;
      t.x.last_rows = 0;
      t.seg_ptrs = nullptr;
      t.nseg = 0;
      t.alpha = (float)((double)j.alpha * (double)j.x.rows / (double)j.x.last_rows);
      if (t.acc) t.acc_beta = 1.f;
      else t.beta = 1.f;
      tail.push_back(t);
      j.x.last_rows = 0;
      if (--j.nseg == 1) {
        j.x.ptr = bases[0];
        j.seg_ptrs = nullptr;
        j.nseg = 0;
      }
    }
    int rc = update_group(head.data(), n, workspace, workspace_bytes, stream);
    if (rc != KFAC_OK) return rc;
    return update_group(tail.data(), (int)tail.size(), workspace, workspace_bytes, stream);
  }
  ConvGeom cg;
  if (n == 1 && gj[0].x.layout != KFAC_ROWMAJOR && job_nseg(gj[0]) > 1 && !conv_geom(gj[0], cg)) {
    // a multi-batch conv job off the image-staged kernel (images too large for LDS):
    // the register-staged kernels read one batch base, so one launch per batch,
    // each adding to what the previous one wrote
    const float* const* bases = reinterpret_cast<const float* const*>(gj[0].seg_ptrs);
    for (int s = 0; s < gj[0].nseg; ++s) {
      kfac_factor_job j = gj[0];
      j.seg_ptrs = nullptr;
      j.nseg = 0;
      j.x.ptr = bases[s];
      if (s > 0) {
        if (j.acc) j.acc_beta = 1.f;
        else j.beta = 1.f;
      }
      const int rc = factor_group(&j, 1, (char*)workspace, workspace_bytes, (hipStream_t)stream);
      if (rc != KFAC_OK) return rc;
    }
    return KFAC_OK;
  }
  int multi = 0, maxseg = 1, total = 0;
  for (int k = 0; k < n; ++k)
    if (job_nseg(gj[k]) > 1) {
      ++multi;
      maxseg = std::max(maxseg, gj[k].nseg);
      total += gj[k].nseg;
    }
  if (total <= KSEG) {
    const int rc = factor_group(gj, n, (char*)workspace, workspace_bytes, (hipStream_t)stream);
    if (rc != KFAC_OK) return rc;
    return KFAC_OK;
  }
  // more batch bases than one launch's kernel arguments hold: rounds of S batches
  // per multi-batch job, each round adding to what the previous ones wrote
  const int S = KSEG / multi;  // >= KSEG / MAXJ = 4
  for (int r = 0; r * S < maxseg; ++r) {
    std::vector<kfac_factor_job> sub;
    for (int k = 0; k < n; ++k) {
      kfac_factor_job j = gj[k];
      if (job_nseg(j) > 1) {
        const int b0 = r * S;
        if (b0 >= j.nseg) continue;
        const float* const* bases = reinterpret_cast<const float* const*>(j.seg_ptrs) + b0;
        j.seg_ptrs = bases;
        j.nseg = std::min(S, j.nseg - b0);
        j.x.ptr = bases[0];
      } else if (r > 0) {
        continue;
      }
      if (r > 0) {
        if (j.acc) j.acc_beta = 1.f;
        else j.beta = 1.f;
      }
      sub.push_back(j);
    }
    const int rc = factor_group(sub.data(), (int)sub.size(), (char*)workspace, workspace_bytes,
                                (hipStream_t)stream);
    if (rc != KFAC_OK) return rc;
  }
  return KFAC_OK;
}

extern "C" int kfac_factor_update(const kfac_factor_job* jobs, int njobs, void* workspace,
                                  size_t workspace_bytes, kfac_stream_t stream) {
  const int rc0 = validate(jobs, njobs);
  if (rc0 != KFAC_OK) return rc0;
  // Launch groups run back to back on the stream, reusing the same workspace.
  std::vector<kfac_factor_job> sorted;
  std::vector<int> order;
  std::vector<std::pair<int, int>> groups;
  launch_groups(jobs, njobs, sorted, order, groups);
  for (const auto& g : groups) {
    const int rc = update_group(sorted.data() + g.first, g.second, workspace, workspace_bytes, stream);
    if (rc != KFAC_OK) return rc;
  }
  return KFAC_OK;
}

extern "C" int kfac_factor_flush(const kfac_factor_job* jobs, int njobs, kfac_stream_t stream) {
  const int rc0 = validate(jobs, njobs);
  if (rc0 != KFAC_OK) return rc0;
  FactorArgs red{};
  int tiles = 0;
  for (int i = 0; i < njobs; ++i) {
    const kfac_factor_job& jb = jobs[i];
    if (!jb.acc) return KFAC_EINVAL;
    FactorJobDev& e = red.job[red.njobs];
    fill_dev(e, jb);
    e.slab = jb.acc;
    e.splits = jb.acc_splits;
    e.sstride = jb.acc_stride > 0 ? jb.acc_stride : jb.acc_splits;
    e.tile_begin = tiles;
    tiles += e.t * (e.t + 1) / 2;
    red.tile_end[red.njobs++] = tiles;
    if (red.njobs == MAXJ || i == njobs - 1) {
      launch_reduce(red, tiles, (hipStream_t)stream);
      KFAC_CHECK_LAUNCH();
      red = FactorArgs{};
      tiles = 0;
    }
  }
  return KFAC_OK;
}

static kfac_operand rowmajor(const float* x, int64_t rows, int64_t cols, int64_t ld, int ones) {
  kfac_operand o{};
  o.ptr = x;
  o.layout = KFAC_ROWMAJOR;
  o.rows = rows;
  o.cols = (int32_t)cols;
  o.ld = ld;
  o.has_ones = ones;
  return o;
}

static int single(const kfac_operand& o, float alpha, float beta, float* F, int64_t ldF, void* ws,
                  size_t wsb, kfac_stream_t s) {
  kfac_factor_job j{};
  j.x = o;
  j.alpha = alpha;
  j.beta = beta;
  j.F = F;
  j.ldF = ldF;
  if (wsb < kfac_factor_workspace_bytes(&j, 1)) return KFAC_EWORKSPACE;
  return kfac_factor_update(&j, 1, ws, wsb, s);
}

extern "C" int kfac_syrk_linear(const float* x, int64_t B, int64_t d, int64_t ldx, int has_ones,
                                float alpha, float beta, float* F, int64_t ldF, void* ws,
                                size_t wsb, kfac_stream_t s) {
  return single(rowmajor(x, B, d, ldx, has_ones ? 1 : 0), alpha, beta, F, ldF, ws, wsb, s);
}

extern "C" int kfac_syrk_conv(const float* x, int64_t B, int C, int H, int W, int kh, int kw,
                              int sh, int sw, int ph, int pw, int has_ones, float alpha, float beta,
                              float* F, int64_t ldF, void* ws, size_t wsb, kfac_stream_t s) {
  if (sh <= 0 || sw <= 0) return KFAC_EINVAL;
  kfac_operand o{};
  o.ptr = x;
  o.layout = KFAC_PATCH;
  o.C = C; o.H = H; o.W = W; o.kh = kh; o.kw = kw; o.sh = sh; o.sw = sw; o.ph = ph; o.pw = pw;
  o.Ho = (H + 2 * ph - kh) / sh + 1;
  o.Wo = (W + 2 * pw - kw) / sw + 1;
  o.L = (int64_t)o.Ho * o.Wo;
  o.sB = (int64_t)C * H * W;
  o.rows = B * o.L;
  o.cols = C * kh * kw;
  o.has_ones = has_ones ? 1 : 0;
  return single(o, alpha, beta, F, ldF, ws, wsb, s);
}

extern "C" int kfac_syrk_convgrad(const float* g, int64_t B, int C, int64_t L, float alpha,
                                  float beta, float* F, int64_t ldF, void* ws, size_t wsb,
                                  kfac_stream_t s) {
  kfac_operand o{};
  o.ptr = g;
  o.layout = KFAC_CHANNEL;
  o.L = L;
  o.sB = (int64_t)C * L;
  o.rows = B * L;
  o.cols = C;
  return single(o, alpha, beta, F, ldF, ws, wsb, s);
}
