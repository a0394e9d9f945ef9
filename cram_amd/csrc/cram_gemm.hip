// cram_gemm.hip — the IE sweep's projection GEMMs on the gfx950 matrix cores, with the MLP activation fused.
//
// out[m, n] = sum_k y[m, k] * x[n, k]: activations y [M, K] and nn.Linear weights x [N, K], both K-contiguous
// (F.linear's layout, the only one the sweep uses).  The reference runs these as transformers' nn.Linear calls
// inside every hooked forward (/root/reference/utils/re_weighting.py:158, :170); here they are the 87 % of the
// head-batched sweep step.
//
// Epilogues
//   CRAM_GEMM_STORE     out = rnd(acc)
//   CRAM_GEMM_SILU_MUL  the LlamaMLP activation on a gate/up weight whose rows are interleaved in blocks of 32
//                       (rows 64j .. 64j+31 = gate rows 32j .. 32j+31, rows 64j+32 .. 64j+63 = the matching up
//                       rows): out[m, f] = rnd(rnd(silu(rnd(g))) * rnd(u)) — transformers' act_fn(gate_proj(x)) *
//                       up_proj(x) on the rounded projections, i.e. cram_silu_mul's arithmetic — so the [M, 2F]
//                       gate/up intermediate never reaches HBM (written once and read back once per layer before).
//
// Structure (one 512-thread workgroup per CU, 256 x 256 output tile, K in 64-deep tiles):
//   * 8 waves as 2 (weight rows, "x") x 4 (activation rows, "y"); a wave owns 128 n x 64 m = 8 x 4 tiles of
//     v_mfma_f32_16x16x32 (x fragments are the A operand, so a lane's accumulator holds 4 consecutive n of one m).
//   * Both operands reach LDS by LDS-DMA (buffer_load_dwordx4 ... lds), two 64 KiB stages.  Rows are 128 B with
//     16-byte chunk c of row r stored at slot c ^ ((r >> 1) & 7): every ds_read_b128 lane group of a fragment
//     read hits 16 distinct slots (conflict-free).  LDS-DMA writes lane-linearly, so the permutation is applied
//     to the per-lane SOURCE address and undone on the read.
//   * A K-tile is 4 phases (quadrants of the wave's tile: 64 n x 32 m x K 64 = 16 MFMAs), each phase a memory
//     interval (fragment reads + one quarter of the staging) and an MFMA interval separated by s_barrier.  Waves
//     4-7 run one interval behind waves 0-3 (one extra barrier up front), so on every SIMD one wave issues MFMAs
//     while its partner issues its reads: the matrix pipe is fed from two waves in turn.
//   * Staging per K-tile in four 16 KiB units (x rows 0-63|128-191, y rows 32-blocks 0,2,4,6, y 1,3,5,7, x
//     64-127|192-255), each issued into the other stage as soon as every wave has consumed the unit it replaces;
//     one counted `s_waitcnt vmcnt(6)` per K-tile retires the next tile while two units of the tile after it stay
//     in flight across the barriers (never vmcnt(0) in the steady loop; raw s_barrier, no __syncthreads fence).
// Requirements (checked by the C-ABI): N % 256 == 0, K % 64 == 0, 16-byte aligned rows; any M >= 1 (rows past M
// read as zeros through the buffer descriptor's range and are not stored).
// Measured at the sweep shape (M = 29,184, bf16 random operands, same-process medians, tools/gemm_probe.py): q/k/v
// 1.00-1.03x hipBLASLt, o_proj 0.97x, gate/up 0.92x, down 0.93x; gate/up + SiLU-mul fused 1.00-1.01x hipBLASLt +
// cram_silu_mul.  The vendor kernel keeps its matrix pipe busy 82 % of the time (4 waves of 128 x 128) against 70 %
// here.  Measured dead ends: one wave per SIMD at 128 x 128 (accumulators pinned in AGPRs by inline
// asm) with LDS-DMA staging 0.81x, with register staging 0.72x, with no staging at all 1.08x (the staging
// instructions in the MFMA wave's own stream are the whole gap); 8 waves software-pipelined with one barrier per
// K-tile 0.85x; a two-phase ping-pong (4 barriers per K-tile) 0.89x.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "../../include/cram_attn.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;

template <typename T> struct GVec;
template <> struct GVec<__bf16> { typedef bf16x8 x8; typedef bf16x4 x4; };
template <> struct GVec<_Float16> { typedef f16x8 x8; typedef f16x4 x4; };

__device__ __forceinline__ f32x4 mfma16(const u32x4& a, const u32x4& b, const f32x4& c, __bf16) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0,
                                                 0, 0);
}
__device__ __forceinline__ f32x4 mfma16(const u32x4& a, const u32x4& b, const f32x4& c, _Float16) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0,
                                                0);
}

// round to the element type and back (the model-dtype rounding transformers applies between ops).  Not as
// (float)(T)x: the compiler folds that pair away in some contexts (cram_fused.hip measured 1-ulp RoPE mismatches on
// ROCm 7.2, and so did the RoPE epilogue here), so bf16 rounds by integer RNE and fp16's hardware conversion is
// pinned in a register.  Inputs are finite.
template <typename T> __device__ __forceinline__ float rnd(float x);
template <> __device__ __forceinline__ float rnd<__bf16>(float x) {
  const unsigned u = __float_as_uint(x);
  return __uint_as_float((u + 0x7FFFu + ((u >> 16) & 1u)) & 0xFFFF0000u);
}
template <> __device__ __forceinline__ float rnd<_Float16>(float x) {
  unsigned short b = __builtin_bit_cast(unsigned short, (_Float16)x);
  asm volatile("" : "+v"(b));
  return (float)__builtin_bit_cast(_Float16, b);
}

constexpr int BM = 256;            // activation rows per tile (y)
constexpr int BN = 256;            // weight rows per tile (x)
constexpr int BK = 64;             // K per tile: 128-byte LDS rows
constexpr int ROWB = BK * 2;       // bytes per LDS row
constexpr int IMG = 256 * ROWB;    // 32 KiB: one operand's image of one K-tile
constexpr int STAGE = 2 * IMG;     // x image | y image
constexpr int LDS_BYTES = 2 * STAGE;

// internal epilogue of the split-K form: fp32 partial sums of one K range, combined by gemm_combine_kernel
constexpr int EPI_PARTIAL = 100;
// internal epilogue of cram_gemm_residual: out = rnd(res + rnd(acc)), the decoder layer's residual add
constexpr int EPI_RESIDUAL = 101;
// internal epilogue of cram_gemm_rope (4-wave kernel only): the q | k | v projection with cram_rope_split's RoPE
constexpr int EPI_ROPE = 102;

struct GemmParams {
  const void* x; int64_t ldx;      // weights [N, K]
  const void* y; int64_t ldy;      // activations [M, K]
  void* out; int64_t ldo;          // [M, N] (store) or [M, N / 2] (silu-mul); EPI_PARTIAL: fp32 [splits][M][N]
  const void* res; int64_t ldr;    // EPI_RESIDUAL: the residual stream [M, N] (may be out itself)
  // EPI_ROPE (head dim 128; a wave's 128 output columns are one head): see cram_gemm_rope in cram_attn.h
  const void* cos_t; const void* sin_t; int64_t tab_rs;
  const int64_t* pos; const int64_t* dst_b; int64_t pos0;
  void* kout; void* vout; int64_t kv_bs, kv_hs, kv_rs;
  int rows, T, hq, hkv, kv_row0, keep_k;
  int M, N, K;
  int ntm, ntn, nblocks;
  int splits, kts;                 // split-K: K ranges per output tile, K-tiles per range (K = splits * kts * BK)
  int raster;                      // gemm_w4_kernel tile order (tile_of_w4); 0 = the default
};

__device__ __forceinline__ void barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// Tile order: bijective XCD remap (each XCD a contiguous run of work ids), then groups of 8 weight tiles with the
// activation tiles innermost, so the 32 workgroups an XCD runs at once share 4 y and 8 x panels.
__device__ __forceinline__ void tile_of(const GemmParams& p, int bid, int& tm, int& tn) {
  const int xcd = bid & 7, q8 = p.nblocks >> 3, r8 = p.nblocks & 7;
  const int wid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  constexpr int GN = 8;
  const int grp = wid / (GN * p.ntm);
  const int gw = min(GN, p.ntn - grp * GN);
  const int rem = wid - grp * GN * p.ntm;
  tn = grp * GN + rem % gw;
  tm = rem / gw;
}

// Epilogue shared by the kernels: lane (j, g) holds acc[a][b][i] = out[m + 16 b][n + 16 a + i] with
// m = tile row + j, n = tile column + 4 g (NA x-tiles of 16 weight rows, NB y-tiles of 16 activation rows).
template <typename T, int EPI, int NA, int NB>
__device__ __forceinline__ void store_tile(const f32x4 (&acc)[NA][NB], const GemmParams& p, int m, int n) {
  using V4 = typename GVec<T>::x4;
  T* ob = static_cast<T*>(p.out);
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const int mb = m + 16 * b;
    if (mb < p.M) {
#pragma unroll
      for (int a = 0; a < NA; ++a) {
        if constexpr (EPI == EPI_PARTIAL) {
          *reinterpret_cast<f32x4*>(static_cast<float*>(p.out) + (int64_t)mb * p.N + n + 16 * a) = acc[a][b];
        } else if constexpr (EPI == CRAM_GEMM_STORE) {
          V4 v;
#pragma unroll
          for (int i = 0; i < 4; ++i) v[i] = (T)acc[a][b][i];
          *reinterpret_cast<V4*>(ob + (int64_t)mb * p.ldo + n + 16 * a) = v;
        } else if constexpr (EPI == EPI_RESIDUAL) {
          const V4 r = *reinterpret_cast<const V4*>(static_cast<const T*>(p.res) + (int64_t)mb * p.ldr + n + 16 * a);
          V4 v;
#pragma unroll
          for (int i = 0; i < 4; ++i) v[i] = (T)((float)r[i] + rnd<T>(acc[a][b][i]));
          *reinterpret_cast<V4*>(ob + (int64_t)mb * p.ldo + n + 16 * a) = v;
        } else if ((a & 2) == 0) {
          // gate tiles a = 0, 1 (mod 4) and their up tiles a + 2 (weight rows interleaved in blocks of 32): the gate
          // column n' = n + 16 a is output column f = 32 * (n' / 64) + n' % 64
          const int ng = n + 16 * a;
          const int f = 32 * (ng >> 6) + (ng & 63);
          V4 v;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float g = rnd<T>(acc[a][b][i]), u = rnd<T>(acc[a + 2][b][i]);
            const float sg = rnd<T>(g / (1.0f + expf(-g)));
            v[i] = (T)(sg * u);
          }
          *reinterpret_cast<V4*>(ob + (int64_t)mb * p.ldo + f) = v;
        }
      }
    }
  }
}

template <typename T, int EPI>
__global__ __launch_bounds__(512) void gemm_tn_kernel(GemmParams p) {
  __shared__ __attribute__((aligned(1024))) char smem[LDS_BYTES];

  int tm, tn, ks = 0;
  GemmParams pp = p;
  if constexpr (EPI == EPI_PARTIAL) {
    // split-K: bid = tile * splits + ks, so the workgroups of one K range (which read the same activation columns)
    // share an XCD under round-robin dispatch when splits is a multiple of 8
    const int tile = blockIdx.x / p.splits;
    ks = blockIdx.x - tile * p.splits;
    tm = tile % p.ntm;
    tn = tile / p.ntm;
    pp.out = static_cast<float*>(p.out) + (int64_t)ks * p.M * p.N;
  } else {
    tile_of(p, blockIdx.x, tm, tn);
  }
  const int n0 = tn * BN, m0 = tm * BM;
  const int k0 = ks * p.kts * BK, kc = p.kts * BK;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wx = wave >> 2, wy = wave & 3;

  // buffer descriptors: x tile rows n0.., y tile rows m0.., columns k0..k0+kc.  Every row offset lives in the
  // per-lane voffset, the only part the range check covers: a y row at or past M has voffset >= the record count
  // (ldy >= kc) and reads zeros; soffset carries only the K-tile offset inside the row.
  const T* xb = static_cast<const T*>(p.x) + (int64_t)n0 * p.ldx + k0;
  const T* yb = static_cast<const T*>(p.y) + (int64_t)m0 * p.ldy + k0;
  const int yrows = min(BM, p.M - m0);
  const auto xsrd = __builtin_amdgcn_make_buffer_rsrc((void*)xb, (short)0, (int)((BN - 1) * p.ldx * 2 + kc * 2),
                                                      0x00020000);
  const auto ysrd = __builtin_amdgcn_make_buffer_rsrc((void*)yb, (short)0, (int)((yrows - 1) * p.ldy * 2 + kc * 2),
                                                      0x00020000);

  // LDS-DMA: unit u, instruction i of this wave writes 8 rows (1 KiB) starting at tile row R(u, 2*wave + i);
  // lane L fetches row R + L/8, chunk (L%8) ^ swz(row)
  const int lr = lane >> 3, ls = lane & 7;
  uint32_t vx[2], vy[2][2];
  int rx[2], ry[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int q = 2 * wave + i;
    rx[i] = q < 8 ? 8 * q : 128 + 8 * (q - 8);                // x_lo unit rows (x_hi: +64)
    ry[i] = (q >> 2) * 64 + 8 * (q & 3);                      // y_lo unit rows (y_hi: +32)
    const int xr = rx[i] + lr;
    vx[i] = (uint32_t)(xr * p.ldx * 2 + ((ls ^ ((xr >> 1) & 7)) * 16));
#pragma unroll
    for (int hi = 0; hi < 2; ++hi) {
      const int yr = ry[i] + 32 * hi + lr;                    // (yr >> 1) & 7 is the same for yr and yr + 32
      vy[i][hi] = (uint32_t)(yr * p.ldy * 2 + ((ls ^ ((yr >> 1) & 7)) * 16));
    }
  }
  const int xhi_off = (int)(64 * p.ldx * 2);
  char* const sbase = smem;
  auto stage_x = [&](int t, int hi) {          // x_lo (hi = 0) or x_hi (hi = 1) of K-tile t
    char* img = sbase + (t & 1) * STAGE;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xsrd, (lds_void*)(img + (rx[i] + 64 * hi) * ROWB), 16, (int)vx[i],
                                               t * ROWB + hi * xhi_off, 0, 0);
  };
  auto stage_y = [&](int t, int hi) {
    char* img = sbase + (t & 1) * STAGE + IMG;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ysrd, (lds_void*)(img + (ry[i] + 32 * hi) * ROWB), 16,
                                               (int)vy[i][hi], t * ROWB, 0, 0);
  };

  // fragment reads: lane (r = lane & 15, g = lane >> 4) reads row r of a 16-row tile, k chunk 4 ks + g
  const int fr = lane & 15, fg = lane >> 4;
  uint32_t foff[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) foff[ks] = (uint32_t)(fr * ROWB + (((4 * ks + fg) ^ (fr >> 1)) * 16));
  const int xrow0 = wx * 128, yrow0 = wy * 64;

  f32x4 acc[8][4];
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  u32x4 xf[4][2], ylo[2][2], yhi[2][2];   // [tile][ks]
  auto read_x = [&](const char* img, int h) {
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        xf[a][ks] = *reinterpret_cast<const u32x4*>(img + (xrow0 + 64 * h + 16 * a) * ROWB + foff[ks]);
  };
  auto read_y = [&](const char* img, int h, u32x4 (&yf)[2][2]) {
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        yf[b][ks] = *reinterpret_cast<const u32x4*>(img + IMG + (yrow0 + 32 * h + 16 * b) * ROWB + foff[ks]);
  };
  auto mma = [&](int h, int yh, const u32x4 (&yf)[2][2]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
          acc[4 * h + a][2 * yh + b] = mfma16(xf[a][ks], yf[b][ks], acc[4 * h + a][2 * yh + b], T{});
    __builtin_amdgcn_s_setprio(0);
  };

  const int nt = p.kts;
  // prologue: all of tile 0, and tile 1 except its x_hi unit (issued in tile 0's first phase)
  stage_x(0, 0); stage_y(0, 0); stage_y(0, 1); stage_x(0, 1);
  if (nt > 1) {
    stage_x(1, 0); stage_y(1, 0); stage_y(1, 1);
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  barrier();
  if (wx == 1) barrier();   // waves 4-7 run one interval behind

  // one K-tile: S1 = a tile t+1 exists (stage its x_hi, wait for it), S2 = a tile t+2 exists (stage 3 units)
  auto ktile = [&](int t, auto s1c, auto s2c) {
    constexpr bool S1 = decltype(s1c)::value, S2 = decltype(s2c)::value;
    const char* img = sbase + (t & 1) * STAGE;
    // phase 0: x rows 0-63 of the wave, y rows 0-31
    read_x(img, 0);
    read_y(img, 0, ylo);
    if constexpr (S1) stage_x(t + 1, 1);
    barrier();
    mma(0, 0, ylo);
    barrier();
    // phase 1: y rows 32-63
    read_y(img, 1, yhi);
    barrier();
    mma(0, 1, yhi);
    barrier();
    // phase 2: x rows 64-127 (x_lo and y_lo of this stage were consumed in phase 0: restage them for t+2)
    read_x(img, 1);
    if constexpr (S2) { stage_x(t + 2, 0); stage_y(t + 2, 0); }
    barrier();
    mma(1, 1, yhi);
    barrier();
    // phase 3: no reads; y_hi (consumed in phase 1) restaged for t+2, then tile t+1 retired
    if constexpr (S2) {
      stage_y(t + 2, 1);
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    } else if constexpr (S1) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    barrier();
    mma(1, 0, ylo);
    barrier();
  };
  using TT = std::integral_constant<bool, true>;
  using FF = std::integral_constant<bool, false>;
  int t = 0;
  for (; t + 2 < nt; ++t) ktile(t, TT{}, TT{});
  if (t + 1 < nt) { ktile(t, TT{}, FF{}); ++t; }
  ktile(t, FF{}, FF{});
  if (wx == 0) barrier();   // equal barrier counts for both halves

  // epilogue: lane (j, g) holds acc[a][b][i] = out[m0 + yrow0 + 16 b + j][n0 + xrow0 + 16 a + 4 g + i]
  store_tile<T, EPI, 8, 4>(acc, pp, m0 + yrow0 + fr, n0 + xrow0 + 4 * fg);
}

// ---------------------------------------------------------------------------------------------------------------
// gemm_w4_kernel: 4 waves (one per SIMD), 128 x 128 outputs per wave in a[0:255], the hand-placed stream of
// tools/gen_gemm_w4.py (gemm_w4_loop.inc): every fragment read, LDS-DMA piece, barrier and counter wait sits in a gap
// between two MFMAs, three barriers per 64-deep K-tile, prefetch one tile ahead through a two-stage LDS ring.  The
// shape of the vendor's 256 x 256 x 64 kernel (the one hipBLASLt picks for the sweep's projections), with this
// library's epilogues.  bf16 / fp16, K-tiles per range >= 2.
// ---------------------------------------------------------------------------------------------------------------
#include "gemm_w4_loop.inc"

constexpr int W4_LDS = 2 * 65536;              // two stages of (weight image 32 KiB | activation image 32 KiB)
#ifdef CRAM_W4_STAMPS
__device__ unsigned* g_w4_stamps;              // [block][wave][5] (diagnostic build only)
#endif

#define CRAM_V128_255_CLOBBERS                                                                                       \
  "v128", "v129", "v130", "v131", "v132", "v133", "v134", "v135", "v136", "v137", "v138", "v139", "v140", "v141",    \
  "v142", "v143", "v144", "v145", "v146", "v147", "v148", "v149", "v150", "v151", "v152", "v153", "v154", "v155",    \
  "v156", "v157", "v158", "v159", "v160", "v161", "v162", "v163", "v164", "v165", "v166", "v167", "v168", "v169",    \
  "v170", "v171", "v172", "v173", "v174", "v175", "v176", "v177", "v178", "v179", "v180", "v181", "v182", "v183",    \
  "v184", "v185", "v186", "v187", "v188", "v189", "v190", "v191", "v192", "v193", "v194", "v195", "v196", "v197",    \
  "v198", "v199", "v200", "v201", "v202", "v203", "v204", "v205", "v206", "v207", "v208", "v209", "v210", "v211",    \
  "v212", "v213", "v214", "v215", "v216", "v217", "v218", "v219", "v220", "v221", "v222", "v223", "v224", "v225",    \
  "v226", "v227", "v228", "v229", "v230", "v231", "v232", "v233", "v234", "v235", "v236", "v237", "v238", "v239",    \
  "v240", "v241", "v242", "v243", "v244", "v245", "v246", "v247", "v248", "v249", "v250", "v251", "v252", "v253",    \
  "v254", "v255"
#define CRAM_A_CLOBBERS_10(b)                                                                                        \
  "a" #b "0", "a" #b "1", "a" #b "2", "a" #b "3", "a" #b "4", "a" #b "5", "a" #b "6", "a" #b "7", "a" #b "8",       \
  "a" #b "9"
// a0..a255 spelled out (the clobbers size the kernel's accumulator file)
#define CRAM_A256_CLOBBERS                                                                                           \
  "a0", "a1", "a2", "a3", "a4", "a5", "a6", "a7", "a8", "a9", CRAM_A_CLOBBERS_10(1), CRAM_A_CLOBBERS_10(2),          \
  CRAM_A_CLOBBERS_10(3), CRAM_A_CLOBBERS_10(4), CRAM_A_CLOBBERS_10(5), CRAM_A_CLOBBERS_10(6), CRAM_A_CLOBBERS_10(7),  \
  CRAM_A_CLOBBERS_10(8), CRAM_A_CLOBBERS_10(9), CRAM_A_CLOBBERS_10(10), CRAM_A_CLOBBERS_10(11),                      \
  CRAM_A_CLOBBERS_10(12), CRAM_A_CLOBBERS_10(13), CRAM_A_CLOBBERS_10(14), CRAM_A_CLOBBERS_10(15),                    \
  CRAM_A_CLOBBERS_10(16), CRAM_A_CLOBBERS_10(17), CRAM_A_CLOBBERS_10(18), CRAM_A_CLOBBERS_10(19),                    \
  CRAM_A_CLOBBERS_10(20), CRAM_A_CLOBBERS_10(21), CRAM_A_CLOBBERS_10(22), CRAM_A_CLOBBERS_10(23),                    \
  CRAM_A_CLOBBERS_10(24), "a250", "a251", "a252", "a253", "a254", "a255"

template <int N, typename F, int I = 0>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<N, F, I + 1>(static_cast<F&&>(f));
  }
}

template <int A>
__device__ __forceinline__ f32x4 acc4() {      // accumulator tile a[A .. A + 3]
  f32x4 v;
  asm volatile("v_accvgpr_read_b32 %0, a[%c4]\n\tv_accvgpr_read_b32 %1, a[%c4+1]\n\t"
               "v_accvgpr_read_b32 %2, a[%c4+2]\n\tv_accvgpr_read_b32 %3, a[%c4+3]"
               : "=v"(v[0]), "=v"(v[1]), "=v"(v[2]), "=v"(v[3]) : "i"(A));
  return v;
}

__device__ __forceinline__ u32x4 w4_srd(const void* base, uint32_t bytes) {
  const uint64_t a = (uint64_t)(uintptr_t)base;
  u32x4 d;
  d[0] = __builtin_amdgcn_readfirstlane((uint32_t)a);
  d[1] = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32) & 0xFFFFu);
  d[2] = __builtin_amdgcn_readfirstlane(bytes);
  d[3] = 0x00020000u;
  return d;
}

// tile order of the 4-wave kernel: the XCD-bijective remap of tile_of, then groups of 8 weight tiles (activation
// tiles innermost) or of 8 activation tiles (weight tiles innermost); measured alternatives (r04, tools/gemm_ab_knob.py):
// groups of 16 weight tiles 0.92-0.95x, no XCD remap 0.86-0.95x
__device__ __forceinline__ int2 tile_of_w4(const GemmParams& p, int bid) {     // (tm, tn)
  const int xcd = bid & 7, q8 = p.nblocks >> 3, r8 = p.nblocks & 7;
  const int wid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  constexpr int G = 8;
  const bool by_m = p.raster == 2;               // groups of 8 activation tiles, weight tiles innermost
  const int nmaj = by_m ? p.ntm : p.ntn, nmin = by_m ? p.ntn : p.ntm;
  const int grp = wid / (G * nmin);
  const int gw = min(G, nmaj - grp * G);
  const int rem = wid - grp * G * nmin;
  const int major = grp * G + rem % gw, minor = rem / gw;
  return by_m ? make_int2(major, minor) : make_int2(minor, major);
}

template <typename T, int EPI>
__global__ __launch_bounds__(256, 1) void gemm_w4_kernel(GemmParams p) {
  __shared__ __attribute__((aligned(1024))) char smem[W4_LDS];
  const int2 tt = tile_of_w4(p, blockIdx.x);
  const int tm = tt.x, tn = tt.y;
  const int n0 = tn * BN, m0 = tm * BM;
  const int kc = p.kts * BK;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wn = wave & 1, wm = wave >> 1;

  const T* xb = static_cast<const T*>(p.x) + (int64_t)n0 * p.ldx;
  const T* yb = static_cast<const T*>(p.y) + (int64_t)m0 * p.ldy;
  const int yrows = min(BM, p.M - m0);
  // rows live in the per-lane voffset (range-checked: a row at or past M reads zeros), the K-tile in soffset
  u32x4 sx = w4_srd(xb, (uint32_t)((BN - 1) * p.ldx * 2 + kc * 2));
  u32x4 sy = w4_srd(yb, (uint32_t)((yrows - 1) * p.ldy * 2 + kc * 2));
  // LDS-DMA piece i of this wave: image rows 32 i + 8 wave .. +7 (the 4 waves' i-th pieces cover 32 adjacent rows);
  // lane L fetches row + L / 8, chunk (L % 8) ^ swz(row)
  uint32_t vx[8], vy[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int row = 32 * i + 8 * wave + (lane >> 3);
    const int c = (lane & 7) ^ ((row >> 1) & 7);
    vx[i] = (uint32_t)(row * p.ldx * 2 + c * 16);
    vy[i] = (uint32_t)(row * p.ldy * 2 + c * 16);
  }
  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)smem;
  uint32_t mx = __builtin_amdgcn_readfirstlane(lds0 + 1024 * wave);
  uint32_t my = __builtin_amdgcn_readfirstlane(lds0 + 32768 + 1024 * wave);
  // K offset of the next tile to stage (soffset); kend wraps it (the generated loop supports a rotated K start: a
  // staggered start per workgroup measured 0.97-0.99x, r04, so every workgroup starts at tile 0)
  uint32_t so = 0;
  const uint32_t kend = (uint32_t)(p.kts * ROWB);
  // fragment reads: lane (r = lane & 15, g = lane >> 4) reads row r of a 16-row fragment, k chunk 4 ks + g
  const int fr = lane & 15, fg = lane >> 4;
  uint32_t rx0 = lds0 + (128 * wn + fr) * ROWB + ((fg ^ (fr >> 1)) * 16);
  uint32_t rx1 = lds0 + (128 * wn + fr) * ROWB + (((4 + fg) ^ (fr >> 1)) * 16);
  uint32_t ry0 = lds0 + 32768 + (128 * wm + fr) * ROWB + ((fg ^ (fr >> 1)) * 16);
  uint32_t ry1 = lds0 + 32768 + (128 * wm + fr) * ROWB + (((4 + fg) ^ (fr >> 1)) * 16);
  uint32_t n = (uint32_t)(p.kts - 2);
  uint32_t keep;
#define CRAM_W4_ASM(LOOP, TY)                                                                                        \
  asm volatile("s_mov_b32 %[keep], m0\n\t"                                                                           \
               "v_accvgpr_write_b32 a0, 0\n\t.set cram_w4i, 1\n\t.rept 255\n\t"                                      \
               "v_accvgpr_write_b32 a[cram_w4i], 0\n\t.set cram_w4i, cram_w4i+1\n\t.endr\n\t"                         \
               LOOP(TY)                                                                                              \
               "s_mov_b32 m0, %[keep]"                                                                               \
               : [keep] "=&s"(keep), [rx0] "+v"(rx0), [rx1] "+v"(rx1), [ry0] "+v"(ry0), [ry1] "+v"(ry1),               \
                 [mx] "+s"(mx), [my] "+s"(my), [so] "+s"(so), [n] "+s"(n)                                            \
               : [sx] "s"(sx), [sy] "s"(sy), [kend] "s"(kend), [vx0] "v"(vx[0]), [vx1] "v"(vx[1]), [vx2] "v"(vx[2]), [vx3] "v"(vx[3]), \
                 [vx4] "v"(vx[4]), [vx5] "v"(vx[5]), [vx6] "v"(vx[6]), [vx7] "v"(vx[7]), [vy0] "v"(vy[0]),           \
                 [vy1] "v"(vy[1]), [vy2] "v"(vy[2]), [vy3] "v"(vy[3]), [vy4] "v"(vy[4]), [vy5] "v"(vy[5]),           \
                 [vy6] "v"(vy[6]), [vy7] "v"(vy[7])                                                                  \
               : "memory", "scc", CRAM_V128_255_CLOBBERS, CRAM_A256_CLOBBERS)
#ifndef CRAM_W4_STAMPS
  if constexpr (std::is_same<T, __bf16>::value) CRAM_W4_ASM(CRAM_GEMM_W4_LOOP_A, "bf16");
  else CRAM_W4_ASM(CRAM_GEMM_W4_LOOP_A, "f16");
#else
  // diagnostic build (tools/w4_stamps.hip): the stamped stream, its per-wave cycle sums (B1, B2, B3, whole tiles,
  // tile count) written to g_w4_stamps -- a buffer of its own, never an output element
  uint32_t st0, st1, st2, st3, st4;
  asm volatile("s_mov_b32 %[keep], m0\n\t"
               "v_accvgpr_write_b32 a0, 0\n\t.set cram_w4i, 1\n\t.rept 255\n\t"
               "v_accvgpr_write_b32 a[cram_w4i], 0\n\t.set cram_w4i, cram_w4i+1\n\t.endr\n\t"
               CRAM_GEMM_W4_LOOP_S("bf16")
               "s_mov_b32 m0, %[keep]\n\t"
               "v_mov_b32 %[st0], s80\n\tv_mov_b32 %[st1], s81\n\tv_mov_b32 %[st2], s82\n\t"
               "v_mov_b32 %[st3], s83\n\tv_mov_b32 %[st4], s84"
               : [keep] "=&s"(keep), [rx0] "+v"(rx0), [rx1] "+v"(rx1), [ry0] "+v"(ry0), [ry1] "+v"(ry1),
                 [mx] "+s"(mx), [my] "+s"(my), [so] "+s"(so), [n] "+s"(n), [st0] "=&v"(st0), [st1] "=&v"(st1),
                 [st2] "=&v"(st2), [st3] "=&v"(st3), [st4] "=&v"(st4)
               : [sx] "s"(sx), [sy] "s"(sy), [kend] "s"(kend), [vx0] "v"(vx[0]), [vx1] "v"(vx[1]), [vx2] "v"(vx[2]),
                 [vx3] "v"(vx[3]), [vx4] "v"(vx[4]), [vx5] "v"(vx[5]), [vx6] "v"(vx[6]), [vx7] "v"(vx[7]),
                 [vy0] "v"(vy[0]), [vy1] "v"(vy[1]), [vy2] "v"(vy[2]), [vy3] "v"(vy[3]), [vy4] "v"(vy[4]),
                 [vy5] "v"(vy[5]), [vy6] "v"(vy[6]), [vy7] "v"(vy[7])
               : "memory", "scc", "s80", "s81", "s82", "s83", "s84", "s85", "s86", "s87", "s88", "s89", "s90", "s91",
                 "s92", "s93", "s94", "s95", CRAM_V128_255_CLOBBERS, CRAM_A256_CLOBBERS);
  if (lane == 0) {
    unsigned* o = g_w4_stamps + ((size_t)blockIdx.x * 4 + wave) * 5;
    o[0] = st0; o[1] = st1; o[2] = st2; o[3] = st3; o[4] = st4;
  }
#endif
#undef CRAM_W4_ASM

  // epilogue through LDS (the output stage of the guide's T21: row-contiguous 16-byte stores instead of 64 scattered
  // 8-byte stores per lane -- the 8-byte form left each workgroup a long store-issue tail).  Lane (r, g) holds acc tile
  // (a, b) = out[m + 16 b + r][n + 16 a + 4 g .. +3]; each wave rounds its 128 rows (256 B each, or 128 B of SiLU-mul
  // output) into its own 32 KiB of the (now idle) ring, 8-byte units swizzled by row so a ds_write lane group spreads
  // over the banks, then reads back whole 16-byte row pieces and stores them (EPI_RESIDUAL: plus the residual piece
  // at the same place, all 32 fetched before the staging so their latency hides behind it).
  using V4 = typename GVec<T>::x4;
  using V8 = typename GVec<T>::x8;
  constexpr bool ROWS = EPI != CRAM_GEMM_SILU_MUL;            // one staged row = 128 output columns
  constexpr int RB = ROWS ? 256 : 128;                         // staged bytes per row
  constexpr int LPR = RB / 16;                                 // read-back lanes per row: 16 | 8
  constexpr int RPI = 64 / LPR;                                // rows per read-back instruction: 4 | 8
  constexpr int NRB = 128 / RPI;                               // read-back instructions per wave
  const int cl = lane % LPR, rl = lane / LPR;
  const int64_t col0 = ROWS ? (int64_t)n0 + 128 * wn + 8 * cl : (int64_t)(n0 / 2) + 64 * wn + 8 * cl;
  const int mw = m0 + 128 * wm;                                // the wave's first output row
  // EPI_ROPE: the wave's head (wave-uniform) -- q heads rotate into out, k heads into kout, v heads are copied into
  // vout (with keep_k the k and v heads also stay in out); without kout every head goes to out (q, k rotated)
  const int hidx = (n0 + 128 * wn) >> 7;
  const int kind = EPI != EPI_ROPE ? 0 : (hidx < p.hq ? 0 : (hidx < p.hq + p.hkv ? 1 : 2));
  V8 rv[EPI == EPI_RESIDUAL ? NRB : 1];
  if constexpr (EPI == EPI_RESIDUAL) {
    const T* rb = static_cast<const T*>(p.res);
#pragma unroll
    for (int j = 0; j < NRB; ++j) {
      const int m = mw + RPI * j + rl;
      if (m < p.M) rv[j] = *reinterpret_cast<const V8*>(rb + (int64_t)m * p.ldr + col0);
    }
  }
  __syncthreads();                               // every wave's last fragment reads are done (no LDS-DMA is pending)
  char* const wl = smem + wave * 32768;
  auto swz = [](int row) { return RB == 256 ? (row & 7) << 2 : ((row >> 1) & 3) << 2; };   // unit XOR (bits 2..4)
  static_for<8>([&](auto bi) {
    constexpr int b = decltype(bi)::value;
    const int ml = 16 * b + fr;                  // the lane's row within the wave's 128
    const int sw = swz(ml);
    if constexpr (ROWS) {
      static_for<8>([&](auto ai) {
        constexpr int a = decltype(ai)::value;
        const f32x4 v = acc4<4 * (8 * a + b)>();
        V4 o;
#pragma unroll
        for (int i = 0; i < 4; ++i) o[i] = (T)v[i];
        *reinterpret_cast<V4*>(wl + ml * RB + (((4 * a + fg) ^ sw) * 8)) = o;
      });
    } else {
      // gate tiles a = 0, 1, 4, 5 and their up tiles a + 2 (weight rows interleaved in blocks of 32): the wave's
      // output columns are f = 32 (a >> 2) + 16 (a & 1) + 4 g + i of its 64
      static_for<4>([&](auto ji) {
        constexpr int a = (decltype(ji)::value & 1) + 4 * (decltype(ji)::value >> 1);
        const f32x4 gv = acc4<4 * (8 * a + b)>(), uv = acc4<4 * (8 * (a + 2) + b)>();
        V4 o;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float g = rnd<T>(gv[i]), u = rnd<T>(uv[i]);
          o[i] = (T)(rnd<T>(g / (1.0f + expf(-g))) * u);
        }
        const int unit = 8 * (a >> 2) + 4 * (a & 1) + fg;
        *reinterpret_cast<V4*>(wl + ml * RB + ((unit ^ sw) * 8)) = o;
      });
    }
  });
  // each wave reads back only its own rows: its writes are ordered before its reads (no barrier needed)
  T* ob = static_cast<T*>(p.out);
  if constexpr (EPI == EPI_RESIDUAL) {
#pragma unroll
    for (int j = 0; j < NRB; ++j) {              // fully unrolled: rv stays in registers
      const int ml = RPI * j + rl;
      V8 v = *reinterpret_cast<const V8*>(wl + ml * RB + (((2 * cl) ^ swz(ml)) * 8));
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = (T)((float)rv[j][i] + (float)v[i]);
      if (mw + ml < p.M) *reinterpret_cast<V8*>(ob + (int64_t)(mw + ml) * p.ldo + col0) = v;
    }
  } else if constexpr (EPI == EPI_ROPE) {
    // read-back by rotation pairs: 8 lanes per row, lane c holds columns 8c.. and 64 + 8c.. of the wave's head;
    // rope_kernel's arithmetic on the staged (rounded) projection, x1' = rnd(rnd(x1 c1) + rnd(-x2 s1)),
    // x2' = rnd(rnd(x2 c2) + rnd(x1 s2)), table row pos[m] (or pos0 + m % T).  Rows go in groups of 4
    // instructions whose table / index loads are all issued before the group's first use (one wait per group).
    const bool rot = kind < 2;
    const bool split = p.kout != nullptr;
    const bool to_out = !split || kind == 0 || p.keep_k;        // keep_k: the k / v heads stay in out too
    const bool to_kv = split && kind != 0;
    const int c8 = lane & 7, r8 = lane >> 3;
    T* const kvb = static_cast<T*>(kind == 2 ? p.vout : p.kout) +
                   (int64_t)(hidx - p.hq - (kind == 2 ? p.hkv : 0)) * p.kv_hs + 8 * c8;
    const int64_t colw = (int64_t)n0 + 128 * wn + 8 * c8;
    const T* const cosb = static_cast<const T*>(p.cos_t) + 8 * c8;
    const T* const sinb = static_cast<const T*>(p.sin_t) + 8 * c8;
#pragma unroll 1
    for (int g = 0; g < 4; ++g) {
      int64_t tp[4], kd[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int m = mw + 8 * (4 * g + u) + r8;
        const bool live = m < p.rows;
        tp[u] = !live ? 0 : (p.pos ? p.pos[m] : p.pos0 + (int64_t)(m % p.T));
        kd[u] = 0;
        if (to_kv && live) {
          const int64_t sb = p.dst_b ? p.dst_b[m] : (int64_t)(m / p.T);
          const int64_t t = p.dst_b ? tp[u] : (int64_t)(m % p.T);
          kd[u] = sb * p.kv_bs + (p.kv_row0 + t) * p.kv_rs;
        }
      }
      V8 c1[4], c2[4], s1[4], s2[4];
      if (rot) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          c1[u] = *reinterpret_cast<const V8*>(cosb + tp[u] * p.tab_rs);
          c2[u] = *reinterpret_cast<const V8*>(cosb + tp[u] * p.tab_rs + 64);
          s1[u] = *reinterpret_cast<const V8*>(sinb + tp[u] * p.tab_rs);
          s2[u] = *reinterpret_cast<const V8*>(sinb + tp[u] * p.tab_rs + 64);
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int ml = 8 * (4 * g + u) + r8;
        const int m = mw + ml;
        V8 x1 = *reinterpret_cast<const V8*>(wl + ml * RB + (((2 * c8) ^ swz(ml)) * 8));
        V8 x2 = *reinterpret_cast<const V8*>(wl + ml * RB + (((16 + 2 * c8) ^ swz(ml)) * 8));
        if (rot) {
          V8 o1, o2;
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const float a = (float)x1[i], b = (float)x2[i];
            o1[i] = (T)(rnd<T>(a * (float)c1[u][i]) + rnd<T>(-b * (float)s1[u][i]));
            o2[i] = (T)(rnd<T>(b * (float)c2[u][i]) + rnd<T>(a * (float)s2[u][i]));
          }
          x1 = o1;
          x2 = o2;
        }
        if (to_out && m < p.M) {
          *reinterpret_cast<V8*>(ob + (int64_t)m * p.ldo + colw) = x1;
          *reinterpret_cast<V8*>(ob + (int64_t)m * p.ldo + colw + 64) = x2;
        }
        if (to_kv && m < p.rows) {
          *reinterpret_cast<V8*>(kvb + kd[u]) = x1;
          *reinterpret_cast<V8*>(kvb + kd[u] + 64) = x2;
        }
      }
    }
  } else {
#pragma unroll 4
    for (int j = 0; j < NRB; ++j) {
      const int ml = RPI * j + rl;
      const V8 v = *reinterpret_cast<const V8*>(wl + ml * RB + (((2 * cl) ^ swz(ml)) * 8));
      if (mw + ml < p.M) *reinterpret_cast<V8*>(ob + (int64_t)(mw + ml) * p.ldo + col0) = v;
    }
  }
}

// Split-K combine: out = epilogue(sum over the K ranges of the fp32 partials [splits][M][N], in range order — the
// result does not depend on which workgroup finished first).  One thread per 8 output columns of one row.
//   CRAM_GEMM_STORE         out[m, n] = rnd(sum + bias[n])            (bias optional: F.linear's addmm epilogue)
//   CRAM_GEMM_SILU_MUL_CAT  x = [gate; up] rows (the checkpoint's own layout, F = N / 2):
//                           out[m, f] = rnd(rnd(silu(rnd(g))) * rnd(u)), g = sum[m, f], u = sum[m, F + f]
template <typename T, int EPI>
__global__ __launch_bounds__(256) void gemm_combine_kernel(const float* __restrict__ part, int splits, int M, int N,
                                                           const T* __restrict__ bias, const T* __restrict__ res,
                                                           int64_t ldr, T* __restrict__ out, int64_t ldo) {
  using V4 = typename GVec<T>::x4;
  const int nout = EPI == CRAM_GEMM_SILU_MUL_CAT ? N / 2 : N;
  const unsigned vpr = (unsigned)nout >> 3;
  const unsigned gid = blockIdx.x * 256u + threadIdx.x;      // host guarantees M * vpr < 2^31
  if (gid >= (unsigned)M * vpr) return;
  const int m = (int)(gid / vpr);
  const int c = (int)(gid % vpr) * 8;
  const int64_t pstride = (int64_t)M * N;
  const float* pr = part + (int64_t)m * N + c;
  float a[8], u[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) a[j] = u[j] = 0.f;
  for (int s = 0; s < splits; ++s) {
    const f32x4 a0 = *reinterpret_cast<const f32x4*>(pr + s * pstride);
    const f32x4 a1 = *reinterpret_cast<const f32x4*>(pr + s * pstride + 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) { a[j] += a0[j]; a[4 + j] += a1[j]; }
    if constexpr (EPI == CRAM_GEMM_SILU_MUL_CAT) {
      const f32x4 u0 = *reinterpret_cast<const f32x4*>(pr + s * pstride + nout);
      const f32x4 u1 = *reinterpret_cast<const f32x4*>(pr + s * pstride + nout + 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) { u[j] += u0[j]; u[4 + j] += u1[j]; }
    }
  }
  V4 o0, o1;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float r;
    if constexpr (EPI == CRAM_GEMM_STORE) {
      r = bias ? a[j] + (float)bias[c + j] : a[j];
    } else if constexpr (EPI == EPI_RESIDUAL) {
      r = (float)res[(int64_t)m * ldr + c + j] + rnd<T>(a[j]);
    } else {
      const float g = rnd<T>(a[j]);
      r = rnd<T>(g / (1.0f + expf(-g))) * rnd<T>(u[j]);
    }
    if (j < 4) o0[j] = (T)r; else o1[j - 4] = (T)r;
  }
  T* op = out + (int64_t)m * ldo + c;
  *reinterpret_cast<V4*>(op) = o0;
  *reinterpret_cast<V4*>(op + 4) = o1;
}

inline bool al16(const void* ptr) { return (reinterpret_cast<uintptr_t>(ptr) & 15u) == 0; }

}  // namespace

namespace {

// shared by cram_gemm and cram_gemm_residual: argument checks, then the 4-wave kernel (bf16, >= 2 K-tiles, 16-byte
// output rows) or the 8-wave one
int gemm_launch(GemmParams& p, int epi, int dtype, hipStream_t st) {
  if (!p.y || !p.x || !p.out || p.M <= 0 || p.N <= 0 || p.K <= 0) return CRAM_ERR_INVALID_ARG;
  if (dtype != CRAM_DTYPE_BF16 && dtype != CRAM_DTYPE_F16) return CRAM_ERR_UNSUPPORTED;
  if (p.N % BN != 0 || p.K % BK != 0) return CRAM_ERR_UNSUPPORTED;
  if (!al16(p.y) || !al16(p.x) || !al16(p.out) || (p.ldy & 7) || (p.ldx & 7) || (p.ldo & 3)) return CRAM_ERR_ALIGNMENT;
  const int nout = epi == CRAM_GEMM_SILU_MUL ? p.N / 2 : p.N;
  if (p.ldy < p.K || p.ldx < p.K || p.ldo < nout) return CRAM_ERR_INVALID_ARG;
  // buffer-descriptor extents (one 256-row tile) are 32-bit byte counts
  if ((int64_t)BN * p.ldx * 2 >= (1ll << 31) || (int64_t)BM * p.ldy * 2 >= (1ll << 31)) return CRAM_ERR_UNSUPPORTED;
  p.splits = 1; p.kts = p.K / BK;
  p.ntm = (p.M + BM - 1) / BM;
  p.ntn = p.N / BN;
  const int64_t nb = (int64_t)p.ntm * p.ntn;
  if (nb > 0x7fffffff) return CRAM_ERR_INVALID_ARG;
  p.nblocks = (int)nb;
  const dim3 g(p.nblocks);
  int kv = -1;
  cram_get_knob(CRAM_KNOB_GEMM_VARIANT, &kv);
  // tile order of the 4-wave kernel: groups of 8 activation tiles for short, narrow GEMMs (q/k/v, o_proj: N <= 6144,
  // K <= 4096: 1.02-1.03x the other order), groups of 8 weight tiles otherwise (down_proj: 1.07x; gate/up: equal)
  // (tools/gemm_ab_knob.py, r04); knob 2 forces the activation-tile groups, 1 the weight-tile groups (A/B)
  p.raster = kv == 2 ? 2 : (kv == 1 ? 0 : ((p.N <= 6144 && p.K <= 4096) ? 2 : 0));
  if (epi == EPI_ROPE) {                         // the 4-wave kernel only (the C-ABI checked bf16, kts >= 2)
    hipLaunchKernelGGL((gemm_w4_kernel<__bf16, EPI_ROPE>), g, dim3(256), 0, st, p);
    return hipGetLastError() == hipSuccess ? CRAM_OK : CRAM_ERR_LAUNCH;
  }
  if (dtype == CRAM_DTYPE_BF16 && p.kts >= 2 && (p.ldo & 7) == 0 && kv != 0) {   // (16-byte output rows)
    if (epi == CRAM_GEMM_STORE) hipLaunchKernelGGL((gemm_w4_kernel<__bf16, CRAM_GEMM_STORE>), g, dim3(256), 0, st, p);
    else if (epi == EPI_RESIDUAL) hipLaunchKernelGGL((gemm_w4_kernel<__bf16, EPI_RESIDUAL>), g, dim3(256), 0, st, p);
    else hipLaunchKernelGGL((gemm_w4_kernel<__bf16, CRAM_GEMM_SILU_MUL>), g, dim3(256), 0, st, p);
    return hipGetLastError() == hipSuccess ? CRAM_OK : CRAM_ERR_LAUNCH;
  }
  const dim3 blk(512);
  if (dtype == CRAM_DTYPE_BF16) {
    if (epi == CRAM_GEMM_STORE) hipLaunchKernelGGL((gemm_tn_kernel<__bf16, CRAM_GEMM_STORE>), g, blk, 0, st, p);
    else if (epi == EPI_RESIDUAL) hipLaunchKernelGGL((gemm_tn_kernel<__bf16, EPI_RESIDUAL>), g, blk, 0, st, p);
    else hipLaunchKernelGGL((gemm_tn_kernel<__bf16, CRAM_GEMM_SILU_MUL>), g, blk, 0, st, p);
  } else {
    if (epi == CRAM_GEMM_STORE) hipLaunchKernelGGL((gemm_tn_kernel<_Float16, CRAM_GEMM_STORE>), g, blk, 0, st, p);
    else if (epi == EPI_RESIDUAL) hipLaunchKernelGGL((gemm_tn_kernel<_Float16, EPI_RESIDUAL>), g, blk, 0, st, p);
    else hipLaunchKernelGGL((gemm_tn_kernel<_Float16, CRAM_GEMM_SILU_MUL>), g, blk, 0, st, p);
  }
  return hipGetLastError() == hipSuccess ? CRAM_OK : CRAM_ERR_LAUNCH;
}

}  // namespace

extern "C" int cram_gemm(const void* y, int64_t ldy, const void* x, int64_t ldx, void* out, int64_t ldo, int M, int N,
                         int K, int epilogue, int dtype, cram_stream_t stream) {
  if (epilogue != CRAM_GEMM_STORE && epilogue != CRAM_GEMM_SILU_MUL) return CRAM_ERR_INVALID_ARG;
  GemmParams p{};
  p.x = x; p.ldx = ldx; p.y = y; p.ldy = ldy; p.out = out; p.ldo = ldo;
  p.M = M; p.N = N; p.K = K;
  return gemm_launch(p, epilogue, dtype, (hipStream_t)stream);
}

extern "C" int cram_gemm_residual(const void* y, int64_t ldy, const void* x, int64_t ldx, const void* res,
                                  int64_t ldr, void* out, int64_t ldo, int M, int N, int K, int dtype,
                                  cram_stream_t stream) {
  if (!res || M <= 0 || N <= 0) return CRAM_ERR_INVALID_ARG;
  if (!al16(res) || (ldr & 7) || (ldo & 7)) return CRAM_ERR_ALIGNMENT;
  if (ldr < N) return CRAM_ERR_INVALID_ARG;
  // the residual may be the output itself (every element is read, then written, by the same lane); any other overlap
  // of the two [M][N] spans is rejected
  const char* r0 = static_cast<const char*>(res);
  const char* o0 = static_cast<const char*>(out);
  if (r0 != o0 || ldr != ldo) {
    const int64_t rspan = ((int64_t)(M - 1) * ldr + N) * 2, ospan = ((int64_t)(M - 1) * ldo + N) * 2;
    if (r0 < o0 + ospan && o0 < r0 + rspan) return CRAM_ERR_INVALID_ARG;
  }
  GemmParams p{};
  p.x = x; p.ldx = ldx; p.y = y; p.ldy = ldy; p.out = out; p.ldo = ldo; p.res = res; p.ldr = ldr;
  p.M = M; p.N = N; p.K = K;
  return gemm_launch(p, EPI_RESIDUAL, dtype, (hipStream_t)stream);
}

extern "C" int cram_gemm_rope(const void* y, int64_t ldy, const void* x, int64_t ldx, void* out, int64_t ldo, int M,
                              int K, int rows, int T, int hq, int hkv, int d, const void* cos_t, const void* sin_t,
                              int64_t tab_rs, const int64_t* pos, int pos0, void* kout, void* vout, int64_t kv_bs,
                              int64_t kv_hs,
                              int64_t kv_rs, int kv_row0, const int64_t* dst_b, int keep_k, int dtype,
                              cram_stream_t stream) {
  if (!cos_t || !sin_t || rows < 0 || rows > M || T <= 0 || hq <= 0 || hkv <= 0 || kv_row0 < 0 || pos0 < 0)
    return CRAM_ERR_INVALID_ARG;
  if ((kout == nullptr) != (vout == nullptr) || (dst_b && !pos) || (kout && !dst_b && rows % T != 0))
    return CRAM_ERR_INVALID_ARG;
  if (dtype != CRAM_DTYPE_BF16 || d != 128 || K % BK != 0 || K / BK < 2) return CRAM_ERR_UNSUPPORTED;
  if ((ldo & 7) || (tab_rs & 7) || !al16(cos_t) || !al16(sin_t)) return CRAM_ERR_ALIGNMENT;
  if (kout && ((kv_bs & 7) || (kv_hs & 7) || (kv_rs & 7) || !al16(kout) || !al16(vout))) return CRAM_ERR_ALIGNMENT;
  GemmParams p{};
  p.x = x; p.ldx = ldx; p.y = y; p.ldy = ldy; p.out = out; p.ldo = ldo;
  p.M = M; p.N = (hq + 2 * hkv) * d; p.K = K;
  p.cos_t = cos_t; p.sin_t = sin_t; p.tab_rs = tab_rs; p.pos = pos; p.pos0 = pos0; p.dst_b = dst_b;
  p.kout = kout; p.vout = vout; p.kv_bs = kv_bs; p.kv_hs = kv_hs; p.kv_rs = kv_rs;
  p.rows = rows; p.T = T; p.hq = hq; p.hkv = hkv; p.kv_row0 = kv_row0; p.keep_k = keep_k;
  return gemm_launch(p, EPI_ROPE, dtype, (hipStream_t)stream);
}

extern "C" size_t cram_gemm_splitk_workspace_size(int M, int N, int splits) {
  if (M <= 0 || N <= 0 || splits <= 0) return 0;
  return (size_t)splits * (size_t)M * (size_t)N * sizeof(float);
}

namespace {

// cram_gemm_splitk / cram_gemm_splitk_residual: partial sums of every (tile, K range) on the 8-wave kernel, then the
// range-ordered combine with the epilogue
int splitk_launch(const void* y, int64_t ldy, const void* x, int64_t ldx, void* out, int64_t ldo, int M, int N, int K,
                  int splits, int epi, const void* bias, const void* res, int64_t ldr, void* workspace,
                  size_t ws_bytes, int dtype, hipStream_t st) {
  if (!y || !x || !out || M <= 0 || N <= 0 || K <= 0 || splits <= 0) return CRAM_ERR_INVALID_ARG;
  if (dtype != CRAM_DTYPE_BF16 && dtype != CRAM_DTYPE_F16) return CRAM_ERR_UNSUPPORTED;
  if (N % BN != 0 || K % (BK * splits) != 0) return CRAM_ERR_UNSUPPORTED;
  if (!al16(y) || !al16(x) || !al16(out) || (ldy & 7) || (ldx & 7) || (ldo & 7)) return CRAM_ERR_ALIGNMENT;
  if (bias && (reinterpret_cast<uintptr_t>(bias) & 15u)) return CRAM_ERR_ALIGNMENT;
  const int nout = epi == CRAM_GEMM_SILU_MUL_CAT ? N / 2 : N;
  if (ldy < K || ldx < K || ldo < nout) return CRAM_ERR_INVALID_ARG;
  if ((int64_t)BN * ldx * 2 >= (1ll << 31) || (int64_t)BM * ldy * 2 >= (1ll << 31)) return CRAM_ERR_UNSUPPORTED;
  if (!workspace || ws_bytes < cram_gemm_splitk_workspace_size(M, N, splits)) return CRAM_ERR_WORKSPACE;
  if ((reinterpret_cast<uintptr_t>(workspace) & 15u)) return CRAM_ERR_ALIGNMENT;
  GemmParams p{};
  p.x = x; p.ldx = ldx; p.y = y; p.ldy = ldy; p.out = workspace; p.ldo = N;
  p.M = M; p.N = N; p.K = K;
  p.splits = splits; p.kts = K / (BK * splits); p.raster = 0;
  p.ntm = (M + BM - 1) / BM;
  p.ntn = N / BN;
  const int64_t nb = (int64_t)p.ntm * p.ntn * splits;
  const int64_t nvec = (int64_t)M * (nout / 8);
  if (nb > 0x7fffffff || nvec >= (1ll << 31)) return CRAM_ERR_INVALID_ARG;
  p.nblocks = (int)nb;
  const dim3 gc((unsigned)((nvec + 255) / 256));
  const float* ws = static_cast<const float*>(workspace);
  auto run = [&](auto tag) {
    using T = decltype(tag);
    hipLaunchKernelGGL((gemm_tn_kernel<T, EPI_PARTIAL>), dim3(p.nblocks), dim3(512), 0, st, p);
    const T* b = static_cast<const T*>(bias);
    const T* r = static_cast<const T*>(res);
    T* o = static_cast<T*>(out);
    if (epi == CRAM_GEMM_STORE)
      hipLaunchKernelGGL((gemm_combine_kernel<T, CRAM_GEMM_STORE>), gc, dim3(256), 0, st, ws, splits, M, N, b, r, ldr, o,
                         ldo);
    else if (epi == EPI_RESIDUAL)
      hipLaunchKernelGGL((gemm_combine_kernel<T, EPI_RESIDUAL>), gc, dim3(256), 0, st, ws, splits, M, N, b, r, ldr, o,
                         ldo);
    else
      hipLaunchKernelGGL((gemm_combine_kernel<T, CRAM_GEMM_SILU_MUL_CAT>), gc, dim3(256), 0, st, ws, splits, M, N, b, r,
                         ldr, o, ldo);
  };
  if (dtype == CRAM_DTYPE_BF16) run(__bf16{});
  else run(_Float16{});
  return hipGetLastError() == hipSuccess ? CRAM_OK : CRAM_ERR_LAUNCH;
}

}  // namespace

extern "C" int cram_gemm_splitk(const void* y, int64_t ldy, const void* x, int64_t ldx, void* out, int64_t ldo,
                                int M, int N, int K, int splits, int epilogue, const void* bias, void* workspace,
                                size_t ws_bytes, int dtype, cram_stream_t stream) {
  if (epilogue != CRAM_GEMM_STORE && epilogue != CRAM_GEMM_SILU_MUL_CAT) return CRAM_ERR_INVALID_ARG;
  if (bias && epilogue != CRAM_GEMM_STORE) return CRAM_ERR_INVALID_ARG;
  return splitk_launch(y, ldy, x, ldx, out, ldo, M, N, K, splits, epilogue, bias, nullptr, 0, workspace, ws_bytes,
                       dtype, (hipStream_t)stream);
}

extern "C" int cram_gemm_splitk_residual(const void* y, int64_t ldy, const void* x, int64_t ldx, const void* res,
                                         int64_t ldr, void* out, int64_t ldo, int M, int N, int K, int splits,
                                         void* workspace, size_t ws_bytes, int dtype, cram_stream_t stream) {
  if (!res || M <= 0 || N <= 0) return CRAM_ERR_INVALID_ARG;
  if (!al16(res) || (ldr & 7)) return CRAM_ERR_ALIGNMENT;
  if (ldr < N) return CRAM_ERR_INVALID_ARG;
  const char* r0 = static_cast<const char*>(res);
  const char* o0 = static_cast<const char*>(out);
  if (r0 != o0 || ldr != ldo) {                  // the residual may be out itself; no other overlap
    const int64_t rspan = ((int64_t)(M - 1) * ldr + N) * 2, ospan = ((int64_t)(M - 1) * ldo + N) * 2;
    if (r0 < o0 + ospan && o0 < r0 + rspan) return CRAM_ERR_INVALID_ARG;
  }
  return splitk_launch(y, ldy, x, ldx, out, ldo, M, N, K, splits, EPI_RESIDUAL, nullptr, res, ldr, workspace,
                       ws_bytes, dtype, (hipStream_t)stream);
}
