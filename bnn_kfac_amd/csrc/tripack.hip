// Packed lower triangles of the KFAC factors, for the data-parallel collectives.
//
// The factors are symmetric (A, G) or lower-triangular (L_A, L_G), so a collective
// only needs n(n+1)/2 of the n^2 elements.  kfac_tri_pack gathers the lower triangle
// of every factor of a call into one contiguous buffer (row i of a factor at
// offset + i(i+1)/2, i+1 elements); kfac_tri_unpack writes it back, mirroring the
// upper triangle (symmetric factors, after the all-reduce of the pass) or zeroing it
// (Cholesky factors, after the all-gather of a sharded inversion).
//
// HBM-bound copies.  One workgroup per 64x64 lower tile of one factor; a wave moves
// one 64-element row segment per instruction (256 B coalesced on both sides); the
// mirrored (J, I) tile of an unpack goes through a padded LDS transpose so its rows
// are written coalesced too.
#include "kfac_common.h"

namespace kfac {
namespace {

constexpr int TRI_MAX_JOBS = 16;

struct TriArgs {
  float* F[TRI_MAX_JOBS];
  int64_t ldF[TRI_MAX_JOBS];
  int64_t off[TRI_MAX_JOBS];
  int32_t n[TRI_MAX_JOBS];
  int32_t tile_start[TRI_MAX_JOBS + 1];  // prefix sums of T(T+1)/2 lower tiles
  int32_t njobs;
  int32_t mode;  // unpack: KFAC_TRI_SYMMETRIC / KFAC_TRI_LOWER
  float* packed;
};

__device__ __forceinline__ int find_job(const TriArgs& a, int b) {
  int j = 0;
  while (j + 1 < a.njobs && a.tile_start[j + 1] <= b) ++j;
  return j;
}

__global__ __launch_bounds__(256) void tri_pack_kernel(TriArgs a) {
  const int job = find_job(a, blockIdx.x);
  int ti, tj;
  tri_decode(blockIdx.x - a.tile_start[job], ti, tj);
  const int n = a.n[job];
  const float* F = a.F[job];
  const int64_t ld = a.ldF[job];
  float* out = a.packed + a.off[job];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int j = tj * TILE + lane;
  for (int r = wave; r < TILE; r += 4) {
    const int i = ti * TILE + r;
    if (i < n && j <= i) out[(int64_t)i * (i + 1) / 2 + j] = F[(int64_t)i * ld + j];
  }
}

__global__ __launch_bounds__(256) void tri_unpack_kernel(TriArgs a) {
  __shared__ float t[TILE][TILE + 1];
  const int job = find_job(a, blockIdx.x);
  int ti, tj;
  tri_decode(blockIdx.x - a.tile_start[job], ti, tj);
  const int n = a.n[job];
  float* F = a.F[job];
  const int64_t ld = a.ldF[job];
  const float* in = a.packed + a.off[job];
  const bool sym = a.mode == KFAC_TRI_SYMMETRIC;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int j = tj * TILE + lane;
  // lower part of tile (ti, tj): straight from the packed rows
  for (int r = wave; r < TILE; r += 4) {
    const int i = ti * TILE + r;
    float v = 0.f;
    if (i < n && j <= i) v = in[(int64_t)i * (i + 1) / 2 + j];
    t[r][lane] = v;
    if (i < n && j < n && (ti != tj || j <= i)) F[(int64_t)i * ld + j] = v;
  }
  if (ti == tj && !sym) {
    // zero the strict upper part of the diagonal tile
    for (int r = wave; r < TILE; r += 4) {
      const int i = ti * TILE + r;
      if (i < n && j < n && j > i) F[(int64_t)i * ld + j] = 0.f;
    }
    return;
  }
  __syncthreads();
  // tile (tj, ti): the transpose (symmetric) or zeros (lower-triangular); on the
  // diagonal only its strict upper part
  const int i2 = ti * TILE + lane;  // column of the mirrored tile
  for (int r = wave; r < TILE; r += 4) {
    const int j2 = tj * TILE + r;  // row of the mirrored tile
    if (j2 < n && i2 < n && (ti != tj || i2 > j2)) F[(int64_t)j2 * ld + i2] = sym ? t[lane][r] : 0.f;
  }
}

int tri_launch(const kfac_tri_job* jobs, int njobs, float* packed, int mode, bool unpack,
               hipStream_t s) {
  if (njobs < 0 || (njobs > 0 && (!jobs || !packed))) return KFAC_EINVAL;
  if (unpack && mode != KFAC_TRI_SYMMETRIC && mode != KFAC_TRI_LOWER) return KFAC_EINVAL;
  for (int j0 = 0; j0 < njobs; j0 += TRI_MAX_JOBS) {
    TriArgs a = {};
    a.njobs = 0;
    a.mode = mode;
    a.packed = packed;
    int64_t tiles = 0;
    for (int j = j0; j < njobs && j < j0 + TRI_MAX_JOBS; ++j) {
      const kfac_tri_job& jb = jobs[j];
      if (!jb.F || jb.n < 0 || jb.ldF < jb.n || jb.offset < 0) return KFAC_EINVAL;
      const int64_t T = cdiv(jb.n, TILE);
      a.F[a.njobs] = jb.F;
      a.ldF[a.njobs] = jb.ldF;
      a.off[a.njobs] = jb.offset;
      a.n[a.njobs] = jb.n;
      a.tile_start[a.njobs] = (int32_t)tiles;
      tiles += T * (T + 1) / 2;
      ++a.njobs;
    }
    a.tile_start[a.njobs] = (int32_t)tiles;
    if (tiles == 0) continue;
    if (tiles > INT32_MAX) return KFAC_EINVAL;
    if (unpack)
      tri_unpack_kernel<<<(unsigned)tiles, 256, 0, s>>>(a);
    else
      tri_pack_kernel<<<(unsigned)tiles, 256, 0, s>>>(a);
    KFAC_CHECK_LAUNCH();
  }
  return KFAC_OK;
}

}  // namespace
}  // namespace kfac

extern "C" int kfac_tri_pack(const kfac_tri_job* jobs, int njobs, float* packed, kfac_stream_t stream) {
  return kfac::tri_launch(jobs, njobs, packed, 0, false, (hipStream_t)stream);
}

extern "C" int kfac_tri_unpack(const kfac_tri_job* jobs, int njobs, const float* packed, int mode,
                               kfac_stream_t stream) {
  return kfac::tri_launch(jobs, njobs, const_cast<float*>(packed), mode, true, (hipStream_t)stream);
}
