// cram_attn.hip — credibility-biased causal GQA attention for MI355X (gfx950, CDNA4).
//
// Replaces the reference's dense-mask forward-pre-hook
// (/root/reference/utils/re_weighting.py:36-61, registered at :118-124 and :163-168)
// plus the SDPA call it feeds.  The hook writes bf16(log_fp16(w_j)) into every
// causal-allowed mask entry of the selected heads; here the same value arrives as
// a per-key fp32 bias vector and is added to the fp32 scores inside the kernel.
//
// Kernels
//   prefill_kernel<D>        flash attention, bf16 MFMA v_mfma_f32_32x32x16_bf16,
//                            "swapped" S^T = K.Q^T so each lane owns one query row
//                            (row softmax is lane-local + one permlane32 swap),
//                            O^T += V^T.P^T with P taken straight from the S^T
//                            accumulator registers and V^T read with
//                            ds_read_b64_tr_b16 from a row-major LDS image.
//                            K/V tiles land in double-buffered LDS by LDS-DMA
//                            (buffer_load ... lds, issued one tile ahead, one barrier
//                            per tile); a workgroup = the query heads of one kv head.
//                            V^T reads are inline asm (through the builtin the waitcnt
//                            pass drains the K/V prefetch with vmcnt(0) before PV);
//                            O leaves through LDS as whole-row 16-byte stores.
//   decode_kernel<D,G>       q_len == 1, HBM-bound: 16 lanes per key row (16 B each,
//                            DPP row reductions), all G query heads of a kv head per
//                            workgroup, optional split over keys + combine_kernel.
//   answer_logits_kernel     fp32 dot of hidden rows with gathered lm_head rows.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <atomic>
#include <mutex>

#include <type_traits>

#include "../../include/cram_attn.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) i16x4 lds_i16x4;
typedef __attribute__((address_space(3))) void lds_void;

// s_waitcnt vmcnt(0) expcnt(7) lgkmcnt(15): wait for vector-memory loads only (gfx9 encoding)
constexpr int kWaitVmcnt0 = 0x0F70;
constexpr float kLog2e = 1.4426950408889634f;
constexpr float kNegInf = -__builtin_huge_valf();

__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// element type of q/k/v/o and of the MFMA operands: bf16 (Llama-3, Qwen2) or fp16 (Llama-2 checkpoints,
// loaded with dtype="auto" as the reference does, re_weighting.py:22)
template <typename T> struct Vec;
template <> struct Vec<__bf16> { typedef bf16x8 x8; typedef bf16x4 x4; };
template <> struct Vec<_Float16> { typedef f16x8 x8; typedef f16x4 x4; };
__device__ __forceinline__ f32x16 mfma32x16(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x16 mfma32x16(f16x8 a, f16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ f32x4 mfma16x32(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma16x32(f16x8 a, f16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}
// max / sum over lanes l, l^16, l^32, l^48 (the four 16-lane rows): one permlane16 and one permlane32 swap
__device__ __forceinline__ float quad_max16(float x) {
  auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  x = fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
  auto t = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(t[0]), __uint_as_float(t[1]));
}
__device__ __forceinline__ float quad_sum16(float x) {
  auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  x = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  auto t = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(t[0]) + __uint_as_float(t[1]);
}

// value from lane l^32 combined with own value (lane halves exchanged by one permlane32 swap)
__device__ __forceinline__ float half_max(float x) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
// sum over the LPK-lane group of a key row (LPK = 16 or 8) with DPP lane swaps inside a 16-lane row:
// xor 1, xor 2 (quad_perm), then the half-row and row mirrors pair every quad with the others
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
template <int LPK>
__device__ __forceinline__ float group_sum(float x) {
  x += dpp_mov<0xB1>(x);    // quad_perm [1,0,3,2]
  x += dpp_mov<0x4E>(x);    // quad_perm [2,3,0,1]
  x += dpp_mov<0x141>(x);   // row_half_mirror: lane i <-> 7-i within each 8 lanes
  if constexpr (LPK == 16) x += dpp_mov<0x140>(x);   // row_mirror: lane i <-> 15-i
  return x;
}
__device__ __forceinline__ float half_sum(float x) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// V^T fragment reads by inline asm: through the builtin, the waitcnt pass treats every ds_read_b64_tr_b16 as
// aliasing the pending LDS-DMA and puts vmcnt(0) in front of it, which would drain the K/V prefetch every tile
// (the .s of prefill_kernel shows it before its PV).  The reads of one 32-key block: 16 x 8 bytes, ordered
// (half, db, s2) -> rr[s2 * 8 + db * 2 + half]; the caller waits on lgkmcnt before consuming them.
template <int VSTR, int KB>
__device__ __forceinline__ void tr_reads32(uint32_t a, i16x4 (&rr)[16]) {
#define CRAM_TR(i, s2, db, h)                                                                     \
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2"                                              \
               : "=v"(rr[i]) : "v"(a), "i"((KB * 32 + 16 * (s2) + 8 * (h)) * VSTR + (db) * 64))
  CRAM_TR(0, 0, 0, 0); CRAM_TR(1, 0, 0, 1); CRAM_TR(2, 0, 1, 0); CRAM_TR(3, 0, 1, 1);
  CRAM_TR(4, 0, 2, 0); CRAM_TR(5, 0, 2, 1); CRAM_TR(6, 0, 3, 0); CRAM_TR(7, 0, 3, 1);
  CRAM_TR(8, 1, 0, 0); CRAM_TR(9, 1, 0, 1); CRAM_TR(10, 1, 1, 0); CRAM_TR(11, 1, 1, 1);
  CRAM_TR(12, 1, 2, 0); CRAM_TR(13, 1, 2, 1); CRAM_TR(14, 1, 3, 0); CRAM_TR(15, 1, 3, 1);
#undef CRAM_TR
}

// O^T[dv][q] += V^T[dv][key] . P^T[key][q] for the 32-key block KB of a tile (d = 128; V image of the tile at LDS
// byte address vaddr - this lane's tr-read base): 16 V^T reads issued together, the first 8 MFMAs after lgkmcnt(8)
// (LDS returns in order), the rest after lgkmcnt(0); sched_barrier keeps the MFMAs behind their waits
template <typename T, int VSTR, int KB>
__device__ __forceinline__ void pv_block32(uint32_t vaddr, const f32x16& pk, f32x16 (&oacc)[4]) {
  using V8 = typename Vec<T>::x8;
  V8 pb[2];
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
    for (int j = 0; j < 8; ++j) pb[s2][j] = (T)pk[8 * s2 + j];
  i16x4 rr[16];
  tr_reads32<VSTR, KB>(vaddr, rr);
  asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int db = 0; db < 4; ++db)   // whole-vector bit casts (per-element extraction of tr results miscompiles)
    oacc[db] = mfma32x16(__builtin_bit_cast(V8, __builtin_shufflevector(rr[2 * db], rr[2 * db + 1], 0, 1, 2, 3, 4, 5,
                                                                        6, 7)), pb[0], oacc[db]);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int db = 0; db < 4; ++db)
    oacc[db] = mfma32x16(__builtin_bit_cast(V8, __builtin_shufflevector(rr[8 + 2 * db], rr[9 + 2 * db], 0, 1, 2, 3,
                                                                        4, 5, 6, 7)), pb[1], oacc[db]);
}

// Epilogue of the prefill kernels: the wave's 32 output rows (lane (r, hh) holds row r's columns
// db*32 + 8g + 4hh .. +3) are staged through LDS as model-dtype rows (2D bytes each) and stored as 16-byte
// pieces of whole rows, 4 rows of d = 128 per instruction, instead of 16 scattered 8-byte stores per lane (the
// store tail is issue-bound: MI355X_MICROARCH.md, attention epilogue).  Staging row i is output row first_row + i.
// The 1/l scaling runs on pairs (v_pk_mul_f32; per element the same product), and the stores go through a buffer
// descriptor that ends at the last row < Tq: rows past it are dropped by the range check (no per-row branch, no
// 64-bit address per store), the row offset of store i is a compile-time multiple of the row stride.
template <typename T, int D>
__device__ __forceinline__ void store_o_rows(char* stage, const f32x16 (&oacc)[D / 32], float inv, int r, int hh,
                                             int lane, T* obase, int64_t o_st, int first_row, int Tq) {
  using V4 = typename Vec<T>::x4;
  constexpr int OSTR = D * 2;                  // unpadded rows; the 16-byte pieces are XOR-swizzled by row
  constexpr int PPR = D * 2 / 16;              // 16-byte pieces per row
  constexpr int RPI = 64 / PPR;                // rows per 64-lane store instruction
  const f32x2 iv = {inv, inv};
#pragma unroll
  for (int db = 0; db < D / 32; ++db)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x2 a = f32x2{oacc[db][4 * g], oacc[db][4 * g + 1]} * iv;
      const f32x2 c = f32x2{oacc[db][4 * g + 2], oacc[db][4 * g + 3]} * iv;
      const V4 o4 = {(T)a[0], (T)a[1], (T)c[0], (T)c[1]};
      // piece db*4 + g of row r lands at piece (db*4 + g) ^ (r mod PPR): the 16 rows of a ds_write_b64 lane group
      // spread over the banks (2-way), and the row-contiguous read-back below is conflict-free
      *reinterpret_cast<V4*>(stage + r * OSTR + ((db * 4 + g) ^ (r & (PPR - 1))) * 16 + hh * 8) = o4;
    }
  const int nrows = min(32, Tq - first_row);
  const int ost2 = (int)o_st * 2;
  const auto osrd = __builtin_amdgcn_make_buffer_rsrc((void*)(obase + (int64_t)first_row * o_st), (short)0,
                                                      nrows > 0 ? (nrows - 1) * ost2 + OSTR : 0, 0x00020000);
  const int lr = lane / PPR, pc = lane % PPR;
  const uint32_t rx = (uint32_t)((pc ^ lr) * 16);   // row i*RPI + lr: (row mod PPR) = ((i*RPI) mod PPR) + lr
  const int voff0 = lr * ost2 + pc * 16;
#pragma unroll
  for (int i = 0; i < 32 / RPI; ++i) {
    const u32x4 v = *reinterpret_cast<const u32x4*>(stage + (i * RPI + lr) * OSTR +
                                                    (rx ^ (uint32_t)(((i * RPI) & (PPR - 1)) * 16)));
    __builtin_amdgcn_raw_buffer_store_b128(v, osrd, voff0 + i * RPI * ost2, 0, 0);
  }
}

// Diagnostic build only (tools/stamp_prefill.hip defines CRAM_STAMPS): every wave takes s_memtime at the
// phase boundaries of each tile into registers, accumulates the per-phase deltas and lane 0 writes the
// sums once at the end (no stores inside the loop: CDNA4's vmcnt counts stores, so per-tile stamp stores
// would be waited for by the loop's own vmcnt).  The product library compiles none of it.
#ifdef CRAM_STAMPS
__device__ unsigned long long* g_stamps;   // [nblocks][4 waves][8]: phase sums 0..5, computed tiles
#define CRAM_STAMP(k) st_[k] = __builtin_amdgcn_s_memtime();
#else
#define CRAM_STAMP(k)
#endif

// --------------------------------------------------------------------------------------------
// prefill
// --------------------------------------------------------------------------------------------
struct PrefillParams {
  const void* q; int64_t q_sb, q_sh, q_st;
  const void* k; int64_t k_sb, k_sh, k_st;
  const void* v; int64_t v_sb, v_sh, v_st;
  void* o; int64_t o_sb, o_sh, o_st;
  const float* bias; int64_t bias_sb;
  const uint8_t* enable; int64_t en_sb;
  int B, Hq, Hkv, Tq, S, W, q_pos0;
  float scale_log2;  // softmax scale * log2(e)
  int nqb, nblocks;
  int hp;             // query heads per workgroup (1, 2 or 4; divides the GQA group)
  const int32_t* cu;  // varlen: [B+1] token offsets of packed sequences (q/k/v/o batch strides unused)
  int kv_cache;       // varlen with cached keys: sequence b's keys are rows 0 .. q_pos0 + Tq_b - 1 of k + b k_sb
                      // (a shared prefix of q_pos0 rows, then its own rows); its queries sit at q_pos0 + i
};

template <int D, int BK_ = 64>
struct PrefillCfg {
  static constexpr int BK = BK_;              // keys per tile
  static constexpr int NKB = BK / 32;         // 32-key MFMA blocks per tile
  static constexpr int KSTR = D * 2 + 16;     // K image row stride (bytes): conflict-free ds_read_b128
  static constexpr int VSTR = D * 2 + 64;     // V image row stride (bytes): conflict-free ds_read_b64_tr_b16
  static constexpr int K_BYTES = BK * KSTR;
  static constexpr int V_BYTES = BK * VSTR;
  static constexpr int B_BYTES = BK * 4;
  static constexpr int KCH = (K_BYTES + 1023) / 1024;   // 1 KiB LDS-DMA chunks of the K image
  static constexpr int VCH = (V_BYTES + 1023) / 1024;
  static constexpr int V_OFF = KCH * 1024;              // V image offset in a stage
  static constexpr int B_OFF = V_OFF + VCH * 1024;      // bias row offset in a stage
  static constexpr int STAGE = B_OFF + B_BYTES;
  static constexpr int LDS = 2 * STAGE;
};

template <typename T, int D, int BK = 64, int OCC = 2, int NW = 4>
__global__ __launch_bounds__(64 * NW, OCC) void prefill_kernel(PrefillParams p) {
  using C = PrefillCfg<D, BK>;
  using V8 = typename Vec<T>::x8;
  static_assert(C::LDS >= NW * 32 * D * 2, "O staging rows must fit in the K/V stages");
  __shared__ __attribute__((aligned(16))) char smem[C::LDS];

  // XCD-aware bijective remap: blocks b and b+8 share an XCD, so give each XCD a
  // contiguous run of work ids (all query blocks of a head -> one L2 for its K/V).
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q8 = p.nblocks >> 3, r8 = p.nblocks & 7;
  const int wid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  // a workgroup = hp query heads of ONE kv head (GQA group) x (NW / hp) waves of 32 query rows:
  // every K/V tile staged in LDS feeds hp heads, and waves that share rows finish together
  const int hp = p.hp, rw = NW / hp, BQ = 32 * rw;
  const int nhg = p.Hq / hp;
  const int qi_blk = wid % p.nqb;
  const int bh = wid / p.nqb;
  const int hg = bh % nhg;
  const int b = bh / nhg;
  const int qblk = p.nqb - 1 - qi_blk;  // heaviest (longest causal range) first
  const int G = p.Hq / p.Hkv;
  const int hkv = (hg * hp) / G;

  // per-sequence extent: uniform batch, or packed varlen sequences (cu_seqlens)
  int Tq = p.Tq, S = p.S, q_pos0 = p.q_pos0;
  int64_t tok0 = 0, ktok0 = 0;
  if (p.cu) {
    tok0 = p.cu[b];
    Tq = p.cu[b + 1] - (int)tok0;
    q_pos0 = p.kv_cache ? p.q_pos0 : 0;
    S = q_pos0 + Tq;
    ktok0 = p.kv_cache ? 0 : tok0;
    if (qblk * BQ >= Tq) return;   // whole workgroup exits before any barrier
  }
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform: scalar branches below
  const int r = lane & 31, hh = lane >> 5;
  const int hq = hg * hp + wave % hp;
  const int q_row0 = qblk * BQ + (wave / hp) * 32;
  const int qrow = q_row0 + r;
  const int qpos = q_pos0 + qrow;

  const T* qb = static_cast<const T*>(p.q) + b * p.q_sb + tok0 * p.q_st + hq * p.q_sh;
  const T* kbase = static_cast<const T*>(p.k) + b * p.k_sb + ktok0 * p.k_st + hkv * p.k_sh;
  const T* vbase = static_cast<const T*>(p.v) + b * p.v_sb + ktok0 * p.v_st + hkv * p.v_sh;
  // per-wave head enable; the workgroup stages the bias tile if any of its heads is enabled
  const bool has_bias = (p.bias != nullptr) && (p.enable != nullptr);
  const bool en = has_bias && p.enable[b * p.en_sb + hq] != 0;
  bool en_any = false;
  if (has_bias)
    for (int j = 0; j < hp; ++j) en_any |= p.enable[b * p.en_sb + hg * hp + j] != 0;
  const float* brow = en_any ? p.bias + b * p.bias_sb : nullptr;

  // Q as the B operand of S^T = K.Q^T: lane (r, hh) holds Q[qrow][16ks + 8hh .. +7]
  // through a descriptor that ends at the wave's last row < Tq (rows past it read zeros): no per-row branch, the
  // loads issue back to back
  V8 qf[D / 16];
  {
    const int qrows = min(32, Tq - q_row0);
    const auto qsrd = __builtin_amdgcn_make_buffer_rsrc((void*)(qb + (int64_t)q_row0 * p.q_st), (short)0,
                                                        qrows > 0 ? (int)((qrows - 1) * p.q_st * 2 + D * 2) : 0,
                                                        0x00020000);
    const int qv = r * (int)p.q_st * 2 + 16 * hh;
#pragma unroll
    for (int ks = 0; ks < D / 16; ++ks)
      qf[ks] = __builtin_bit_cast(V8, __builtin_amdgcn_raw_buffer_load_b128(qsrd, qv + 32 * ks, 0, 0));
  }

  const int blk_last_q = min(qblk * BQ + BQ, Tq) - 1;
  const int kv_end = min(S, q_pos0 + blk_last_q + 1);
  const int nt = (kv_end + C::BK - 1) / C::BK;
  const bool wave_live = q_row0 < Tq;
  const int wave_qpos_min = q_pos0 + q_row0;
  const int wave_qpos_max = q_pos0 + min(q_row0 + 31, Tq - 1);

  // K/V/bias staging through buffer descriptors: per-thread byte offsets are loop invariant, the
  // per-tile base and the valid extent live in scalar registers, and the descriptor's range check
  // returns zeros past key S (no per-load VALU address math, no bounds compares).
  // K/V staging by LDS-DMA (buffer_load ... lds): no VGPR staging, no ds_write.  One wave-instruction
  // writes 1 KiB of the padded (K | V) image of a tile = 64 lanes x 16 B; lane p of chunk c fetches
  // the 16 bytes that belong at image offset c*1024 + 16p (a pad slot gets an out-of-range offset, so
  // the descriptor's range check writes zeros there, as it does for rows past key S).
  // chunks of the K image are c = wave + NW i (i < KPW), then those of the V image likewise: only a wave's last chunk
  // of each image can fall past it, so the K-or-V choice is compile-time (a per-chunk runtime choice keeps ~40
  // scalar lane conditions live)
  constexpr int KCH = C::KCH, VCH = C::VCH;
  constexpr int KPW = (KCH + NW - 1) / NW, VPW = (VCH + NW - 1) / NW;
  uint32_t dk[KPW], dv[VPW];
#pragma unroll
  for (int i = 0; i < KPW; ++i) {
    const int x = (wave + NW * i) * 1024 + 16 * lane, row = x / C::KSTR, colb = x % C::KSTR;
    dk[i] = (x < C::K_BYTES && colb < D * 2) ? (uint32_t)(row * p.k_st * 2 + colb) : 0xFFFFFFF0u;
  }
#pragma unroll
  for (int i = 0; i < VPW; ++i) {
    const int x = (wave + NW * i) * 1024 + 16 * lane, row = x / C::VSTR, colb = x % C::VSTR;
    dv[i] = (x < C::V_BYTES && colb < D * 2) ? (uint32_t)(row * p.v_st * 2 + colb) : 0xFFFFFFF0u;
  }
  float bst = 0.f;

  auto gload = [&](int t) {                    // tile t -> LDS buffer t & 1 (asynchronous)
    const int key0 = t * C::BK;
    const int rows_left = S - key0;   // > 0 for every tile of the loop
    const auto ksrd = __builtin_amdgcn_make_buffer_rsrc((void*)(kbase + (int64_t)key0 * p.k_st), (short)0,
                                                        (int)((rows_left - 1) * p.k_st * 2 + D * 2), 0x00020000);
    const auto vsrd = __builtin_amdgcn_make_buffer_rsrc((void*)(vbase + (int64_t)key0 * p.v_st), (short)0,
                                                        (int)((rows_left - 1) * p.v_st * 2 + D * 2), 0x00020000);
    char* base = smem + (t & 1) * C::STAGE;
#pragma unroll
    for (int i = 0; i < KPW; ++i) {
      const int c = wave + NW * i;
      if ((i + 1) * NW <= KCH || c < KCH)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(ksrd, (lds_void*)(base + c * 1024), 16, (int)dk[i], 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < VPW; ++i) {
      const int c = wave + NW * i;
      if ((i + 1) * NW <= VCH || c < VCH)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(vsrd, (lds_void*)(base + C::V_OFF + c * 1024), 16, (int)dv[i], 0, 0,
                                                 0);
    }
    if (en_any && tid < C::BK) {
      const int wl = p.W - key0;
      const auto bsrd = __builtin_amdgcn_make_buffer_rsrc((void*)(brow + key0), (short)0, wl > 0 ? wl * 4 : 0,
                                                          0x00020000);
      bst = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(bsrd, tid * 4, 0, 0));   // scaled in swrite
    }
  };
  auto swrite = [&](int buf) {                 // the bias row (register staged)
    char* base = smem + buf * C::STAGE;
    if (en_any && tid < C::BK) reinterpret_cast<float*>(base + C::B_OFF)[tid] = bst * kLog2e;
  };

  float m = kNegInf, l = 0.f;
  f32x16 oacc[D / 32];
#pragma unroll
  for (int db = 0; db < D / 32; ++db)
#pragma unroll
    for (int e = 0; e < 16; ++e) oacc[db][e] = 0.f;

  // per-lane constant LDS offsets
  const int g16 = lane >> 4, i16 = lane & 15;
  const int tr_key = 4 * (g16 >> 1) + (i16 >> 2);              // + kb*32 + 16s (+8)
  const int tr_col = 16 * (g16 & 1) + 4 * (i16 & 3);            // + db*32

  if (nt > 0) {
    gload(0);
    swrite(0);
  }
  // Q (and the first tile) must be complete on EVERY path into the loop: otherwise the waitcnt pass
  // merges a pending Q load into the loop header and puts vmcnt(0) in front of the first MFMA of
  // every tile, serialising each tile with the next tile's prefetch.
  __builtin_amdgcn_s_waitcnt(kWaitVmcnt0);
  __syncthreads();

#ifdef CRAM_STAMPS
  unsigned long long st_[6] = {}, acc_[7] = {};
#endif
  // One K/V tile with NB 32-key MFMA blocks: C::NKB, or 1 for the workgroup's last tile when its upper 32 keys lie
  // past every row's causal / length limit (kv_end <= key0 + 32: the block would be all -inf; skipping it removes
  // the fully masked MFMAs of half the diagonal tiles).  Score arithmetic on pairs (v_pk_fma_f32): per element the
  // same fma as before; the row sums stay sequential (two interleaved partial sums moved a near-tie answer log-prob
  // across the drop-in's noise-floor bar).
  auto tile = [&](int t, auto nbc) {
    constexpr int NB = decltype(nbc)::value;
    CRAM_STAMP(0)
    if (t + 1 < nt) gload(t + 1);
    const int key0 = t * C::BK;
    if (wave_live && key0 <= wave_qpos_max) {
      const char* base = smem + (t & 1) * C::STAGE;
      f32x16 sacc[C::NKB];
      const f32x16 zero16 = {};
#pragma unroll
      for (int kb = 0; kb < NB; ++kb) {
#pragma unroll
        for (int ks = 0; ks < D / 16; ++ks) {
          const V8 a = *reinterpret_cast<const V8*>(base + (kb * 32 + r) * C::KSTR + (16 * ks + 8 * hh) * 2);
          sacc[kb] = mfma32x16(a, qf[ks], ks == 0 ? zero16 : sacc[kb]);
        }
      }
      // scores (log2 units): scale, credibility bias, causal / length mask.  Wave-uniform split: a tile
      // with no masked key and no bias keeps the raw scores (max of raw scores, then one scaled max:
      // fl(c*s) is monotone in s, so it equals the max of the scaled scores) and folds the scale into
      // the exponent's FMA.
      const float* bl = reinterpret_cast<const float*>(base + C::B_OFF);
      const bool need_mask = (key0 + 32 * NB - 1 > wave_qpos_min) || (key0 + 32 * NB > S);
      const bool plain = !need_mask && !en;
      const f32x2 c2 = {p.scale_log2, p.scale_log2};
      float mx = kNegInf;
      if (plain) {
#pragma unroll
        for (int kb = 0; kb < NB; ++kb)
#pragma unroll
          for (int e = 0; e < 16; ++e) mx = fmaxf(mx, sacc[kb][e]);
        mx *= p.scale_log2;
      } else if (!need_mask) {                                   // biased head, interior tile
        // raw scores stay in sacc: the exponent below is fma(s, c, b - m), which for b == 0 is exactly
        // the plain path's fma(s, c, -m) (a zero bias is bit-identical to no bias)
#pragma unroll
        for (int kb = 0; kb < NB; ++kb) {
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const f32x4 bv = *reinterpret_cast<const f32x4*>(bl + kb * 32 + 8 * g + 4 * hh);
#pragma unroll
            for (int e = 0; e < 4; e += 2) {
              const f32x2 sv = {sacc[kb][4 * g + e], sacc[kb][4 * g + e + 1]};
              const f32x2 v = __builtin_elementwise_fma(sv, c2, f32x2{bv[e], bv[e + 1]});
              mx = fmaxf(mx, fmaxf(v[0], v[1]));
            }
          }
        }
      } else {                                                   // diagonal / ragged tile
        const int lim = min(qpos, S - 1) - key0;
#pragma unroll
        for (int kb = 0; kb < NB; ++kb) {
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            f32x4 bv = {0.f, 0.f, 0.f, 0.f};
            if (en) bv = *reinterpret_cast<const f32x4*>(bl + kb * 32 + 8 * g + 4 * hh);
#pragma unroll
            for (int e = 0; e < 4; e += 2) {
              const f32x2 sv = {sacc[kb][4 * g + e], sacc[kb][4 * g + e + 1]};
              f32x2 v = __builtin_elementwise_fma(sv, c2, f32x2{bv[e], bv[e + 1]});
              // branch-free causal / length mask: key offset in tile vs the lane's last allowed key
              const int col = kb * 32 + 8 * g + 4 * hh + e;
              v[0] = (col > lim) ? kNegInf : v[0];
              v[1] = (col + 1 > lim) ? kNegInf : v[1];
              sacc[kb][4 * g + e] = v[0];
              sacc[kb][4 * g + e + 1] = v[1];
              mx = fmaxf(mx, fmaxf(v[0], v[1]));
            }
          }
        }
      }
      mx = half_max(mx);
      CRAM_STAMP(1)
      const float mnew = fmaxf(m, mx);
      const float muse = (mnew == kNegInf) ? 0.f : mnew;
      const float alpha = fast_exp2(m - muse);
      float rs = 0.f;                         // sequential sum: the previous kernel's rounding, bit for bit
      const f32x2 nm2 = {-muse, -muse};
      if (!plain && !need_mask) {
#pragma unroll
        for (int kb = 0; kb < NB; ++kb)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const f32x4 bv = *reinterpret_cast<const f32x4*>(bl + kb * 32 + 8 * g + 4 * hh);
#pragma unroll
            for (int e = 0; e < 4; e += 2) {
              const f32x2 sv = {sacc[kb][4 * g + e], sacc[kb][4 * g + e + 1]};
              f32x2 v = __builtin_elementwise_fma(sv, c2, f32x2{bv[e], bv[e + 1]} + nm2);
              v[0] = fast_exp2(v[0]);
              v[1] = fast_exp2(v[1]);
              sacc[kb][4 * g + e] = v[0];
              sacc[kb][4 * g + e + 1] = v[1];
              rs += v[0];
              rs += v[1];
            }
          }
      } else {
        const float sc = plain ? p.scale_log2 : 1.f;
        const f32x2 sc2 = {sc, sc};
#pragma unroll
        for (int kb = 0; kb < NB; ++kb) {
#pragma unroll
          for (int e = 0; e < 16; e += 2) {
            const f32x2 sv = {sacc[kb][e], sacc[kb][e + 1]};
            f32x2 v = __builtin_elementwise_fma(sv, sc2, nm2);
            v[0] = fast_exp2(v[0]);
            v[1] = fast_exp2(v[1]);
            sacc[kb][e] = v[0];
            sacc[kb][e + 1] = v[1];
            rs += v[0];
            rs += v[1];
          }
        }
      }
      rs = half_sum(rs);
      CRAM_STAMP(2)
      l = l * alpha + rs;
      m = mnew;
      // the running max rarely moves after the first tiles: skip the O rescale when alpha == 1 on
      // every lane (exact; a wave-uniform branch)
      if (__builtin_amdgcn_ballot_w64(alpha != 1.f)) {
#pragma unroll
        for (int db = 0; db < D / 32; ++db)
#pragma unroll
          for (int e = 0; e < 16; ++e) oacc[db][e] *= alpha;
      }

      // O^T[dv][q] += V^T[dv][key] . P^T[key][q]
      const char* vimg = base + C::V_OFF;
      if constexpr (D == 128) {     // V^T reads by inline asm (tr_reads32): the K/V prefetch stays in flight
        const uint32_t vaddr = (uint32_t)(uintptr_t)(const lds_void*)vimg + (uint32_t)(tr_key * C::VSTR + tr_col * 2);
        pv_block32<T, C::VSTR, 0>(vaddr, sacc[0], oacc);
        if constexpr (NB == 2) pv_block32<T, C::VSTR, 1>(vaddr, sacc[1], oacc);
      } else
#pragma unroll
      for (int kb = 0; kb < NB; ++kb) {
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          V8 pb;
#pragma unroll
          for (int j = 0; j < 8; ++j) pb[j] = (T)sacc[kb][8 * s + j];
          const int key_a = kb * 32 + 16 * s + tr_key;
#pragma unroll
          for (int db = 0; db < D / 32; ++db) {
            const int col = db * 32 + tr_col;
            const i16x4 r1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (lds_i16x4*)(vimg + key_a * C::VSTR + col * 2));
            const i16x4 r2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (lds_i16x4*)(vimg + (key_a + 8) * C::VSTR + col * 2));
            // whole-vector bit cast (per-element extraction of the tr result miscompiles on ROCm 7.2)
            const V8 af = __builtin_bit_cast(V8, __builtin_shufflevector(r1, r2, 0, 1, 2, 3, 4, 5, 6, 7));
            oacc[db] = mfma32x16(af, pb, oacc[db]);
          }
        }
      }
    }
    CRAM_STAMP(3)
#ifdef CRAM_STAMPS
    __builtin_amdgcn_s_waitcnt(kWaitVmcnt0);   // separates the DMA wait from the barrier wait
    CRAM_STAMP(5)
#endif
    if (t + 1 < nt) swrite((t + 1) & 1);
    __syncthreads();
    CRAM_STAMP(4)
#ifdef CRAM_STAMPS
    if (st_[1]) {                                   // a tile this wave computed
      acc_[0] += st_[1] - st_[0]; acc_[1] += st_[2] - st_[1]; acc_[2] += st_[3] - st_[2];
      acc_[3] += st_[5] - st_[3]; acc_[4] += st_[4] - st_[5]; acc_[6] += 1;
    }
    st_[1] = 0;
#endif
  };
  const bool half_last = C::NKB == 2 && nt > 0 && kv_end <= (nt - 1) * C::BK + 32;
  const int nfull = half_last ? nt - 1 : nt;
  for (int t = 0; t < nfull; ++t) tile(t, std::integral_constant<int, C::NKB>{});
  if (half_last) tile(nt - 1, std::integral_constant<int, 1>{});

#ifdef CRAM_STAMPS
  if (lane == 0)
    for (int k = 0; k < 7; ++k) g_stamps[((size_t)wid * 4 + wave) * 8 + k] = acc_[k];
#endif
  // every wave passed the last tile's barrier: the stages are free for the O staging rows
  store_o_rows<T, D>(smem + wave * 32 * (D * 2), oacc, l > 0.f ? 1.f / l : 0.f, r, hh, lane,
                     static_cast<T*>(p.o) + b * p.o_sb + tok0 * p.o_st + hq * p.o_sh, p.o_st, q_row0, Tq);
}

// register-pinned asm helpers of the hand-scheduled prefill (prefill_asm.inc) and the kernel (prefill_x32.inc)
#include "prefill_asm.inc"
// two workgroups per CU, 32 rows per wave, the same hand-ordered stream: prefill_x32_kernel
#include "prefill_x32.inc"

// --------------------------------------------------------------------------------------------
// decode (q_len == 1)
// --------------------------------------------------------------------------------------------
struct DecodeParams {
  const void* q; int64_t q_sb, q_sh;
  const void* k; int64_t k_sb, k_sh, k_st;
  const void* v; int64_t v_sb, v_sh, v_st;
  void* o; int64_t o_sb, o_sh;
  const float* bias; int64_t bias_sb;
  const uint8_t* enable; int64_t en_sb;
  const int32_t* seq_lens;
  int B, Hq, Hkv, S, W;
  float scale_log2;
  float* ws_o;   // [B][Hq][nsplit][D] unnormalised partial outputs (split mode)
  float* ws_ml;  // [B][Hq][nsplit][2]  partial (max, sum)
  int shared;    // keys [0, shared) are equal in every batch row (a shared prompt opening, copied into each row): the
                 // matrix-core body reads them from batch row 0 (one HBM stream for the batch); a multiple of 32
};

template <typename T, int D, int G, int U = 4>   // U: keys per lane group per iteration
__global__ __launch_bounds__(256) void decode_kernel(DecodeParams p) {
  using V8 = typename Vec<T>::x8;
  constexpr int LPK = D / 8;        // lanes per key row (8 elements = 16 B per lane)
  constexpr int KPW = 64 / LPK;     // keys per wave-instruction
  constexpr int STEP = 4 * KPW;     // keys per workgroup per unrolled slot
  __shared__ float red_m[4][G], red_l[4][G];
  __shared__ float red_o[4][G][D];

  const int hkv = blockIdx.x, b = blockIdx.y, split = blockIdx.z, nsplit = gridDim.z;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform: scalar branches below
  const int grp = lane / LPK, li = lane % LPK;

  const int S_b = p.seq_lens ? p.seq_lens[b] : p.S;
  const int chunk = (((S_b + nsplit - 1) / nsplit) + 63) & ~63;
  const int k_begin = split * chunk;
  const int k_end = min(S_b, k_begin + chunk);

  float qv[G][8];
  bool en[G];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const int hq = hkv * G + g;
    const V8 qq = *reinterpret_cast<const V8*>(static_cast<const T*>(p.q) + b * p.q_sb + hq * p.q_sh + li * 8);
#pragma unroll
    for (int j = 0; j < 8; ++j) qv[g][j] = (float)qq[j] * p.scale_log2;
    en[g] = (p.bias != nullptr) && (p.enable != nullptr) && p.enable[b * p.en_sb + hq] != 0;
  }
  const float* brow = p.bias ? p.bias + b * p.bias_sb : nullptr;
  const T* kbase = static_cast<const T*>(p.k) + b * p.k_sb + hkv * p.k_sh + li * 8;
  const T* vbase = static_cast<const T*>(p.v) + b * p.v_sb + hkv * p.v_sh + li * 8;

  float m[G], l[G], acc[G][8];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    m[g] = kNegInf;
    l[g] = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[g][j] = 0.f;
  }

  // K/V rows of the next iteration are loaded while the current one is computed (register double
  // buffer): every wave keeps 2 x U x 2 16-byte loads in flight instead of stalling on each batch
  V8 kn[U], vn[U];
  auto load_keys = [&](int kb0) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int key = kb0 + u * STEP;
      if (key < k_end) {
        kn[u] = *reinterpret_cast<const V8*>(kbase + key * p.k_st);
        vn[u] = *reinterpret_cast<const V8*>(vbase + key * p.v_st);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) { kn[u][j] = (T)0.f; vn[u][j] = (T)0.f; }
      }
    }
  };
  constexpr bool PF = G <= 4;   // larger head groups keep two waves per SIMD instead (VGPR budget)
  if (PF) load_keys(k_begin + wave * KPW + grp);
  for (int key_base = k_begin + wave * KPW + grp; key_base < k_end; key_base += U * STEP) {
    if (!PF) load_keys(key_base);
    V8 kr[U], vr[U];
    bool valid[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      kr[u] = kn[u];
      vr[u] = vn[u];
      valid[u] = key_base + u * STEP < k_end;
    }
    if (PF && key_base + U * STEP < k_end) load_keys(key_base + U * STEP);
    float bias_u[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int key = key_base + u * STEP;
      bias_u[u] = (brow && valid[u] && key < p.W) ? brow[key] * kLog2e : 0.f;
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
      float s[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        float d = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) d += qv[g][j] * (float)kr[u][j];
        d = group_sum<LPK>(d);
        s[u] = valid[u] ? d + (en[g] ? bias_u[u] : 0.f) : kNegInf;
      }
      float mx = s[0];
#pragma unroll
      for (int u = 1; u < U; ++u) mx = fmaxf(mx, s[u]);
      const float mnew = fmaxf(m[g], mx);
      const float muse = (mnew == kNegInf) ? 0.f : mnew;
      const float alpha = fast_exp2(m[g] - muse);
      l[g] *= alpha;
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[g][j] *= alpha;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const float pu = fast_exp2(s[u] - muse);
        l[g] += pu;
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[g][j] += pu * (float)vr[u][j];
      }
      m[g] = mnew;
    }
  }

  // combine the lane groups of this wave (groups differ by lane bits above log2(LPK))
#pragma unroll
  for (int off = LPK; off < 64; off <<= 1) {
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const float mo = __shfl_xor(m[g], off, 64);
      const float lo = __shfl_xor(l[g], off, 64);
      const float mnew = fmaxf(m[g], mo);
      const float muse = (mnew == kNegInf) ? 0.f : mnew;
      const float a0 = fast_exp2(m[g] - muse), a1 = fast_exp2(mo - muse);
      l[g] = l[g] * a0 + lo * a1;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float ao = __shfl_xor(acc[g][j], off, 64);
        acc[g][j] = acc[g][j] * a0 + ao * a1;
      }
      m[g] = mnew;
    }
  }
  if (grp == 0) {
#pragma unroll
    for (int g = 0; g < G; ++g) {
      if (li == 0) { red_m[wave][g] = m[g]; red_l[wave][g] = l[g]; }
#pragma unroll
      for (int j = 0; j < 8; ++j) red_o[wave][g][li * 8 + j] = acc[g][j];
    }
  }
  __syncthreads();
  // combine the 4 waves: thread t handles (g, dim) pairs
  for (int idx = tid; idx < G * D; idx += 256) {
    const int g = idx / D, dd = idx % D;
    float M = kNegInf;
#pragma unroll
    for (int w = 0; w < 4; ++w) M = fmaxf(M, red_m[w][g]);
    const float Muse = (M == kNegInf) ? 0.f : M;
    float L = 0.f, O = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const float a = fast_exp2(red_m[w][g] - Muse);
      L += red_l[w][g] * a;
      O += red_o[w][g][dd] * a;
    }
    const int hq = hkv * G + g;
    if (nsplit == 1) {
      static_cast<T*>(p.o)[b * p.o_sb + hq * p.o_sh + dd] = (T)(L > 0.f ? O / L : 0.f);
    } else {
      const int64_t slot = ((int64_t)(b * p.Hq + hq) * nsplit + split);
      p.ws_o[slot * D + dd] = O;
      if (dd == 0) { p.ws_ml[slot * 2 + 0] = M; p.ws_ml[slot * 2 + 1] = L; }
    }
  }
}

// --------------------------------------------------------------------------------------------
// decode on the matrix cores (GQA groups of 4..16 query heads, d = 128)
// --------------------------------------------------------------------------------------------
// All G query heads of one kv head against 32-key blocks, per wave, with v_mfma_f32_16x16x32:
//   S^T[16 keys][16 q]  = K[16 keys][d] . Q^T[d][16 q]   (A = K rows straight from HBM into VGPRs: lane l loads
//                                                          16 B of key row l&15; B = Q^T held for the whole loop)
//   O^T[16 d][16 q]    += V^T[16 d][32 keys] . P^T[32 keys][16 q]
// Lane l owns query head q = l&15 and keys 4(l>>4)+i (+16) of a block, which is exactly the B-operand slot
// order of the PV product (slots 0-3 = keys 4g..4g+3, 4-7 = keys 16+4g..16+4g+3), so P goes from the score
// registers to the operand by 4 conversions; V^T comes from a per-wave LDS image of the block's V rows
// (register-staged, 288-B rows: the ds_read_b64_tr_b16 of 8 rows x 16 columns hit 64 distinct banks).
// The waves of a workgroup take alternate key blocks and share nothing until the final combine, so the loop has
// no barrier; K/V of the next block are loaded while the current one is computed.  Query heads >= G are zero
// columns.  The VALU kernel spends ~G x 26 instructions per key and lane on the dot products, reductions and
// online softmax: at G = 7 (Qwen2) that body read 2.9 TB/s; here the dot products run on the matrix cores.
template <typename T, int G>
__global__ __launch_bounds__(256, 2) void decode_mfma_kernel(DecodeParams p) {
  constexpr int D = 128;
  constexpr int VSTR = D * 2 + 32;          // V image row stride (bytes)
  constexpr int KB = 32;                    // keys per block
  constexpr int VIMG = KB * VSTR;           // 9216 B per wave
  using V8 = typename Vec<T>::x8;
  static_assert(G <= 16, "one 16-column MFMA tile of query heads");
  __shared__ __attribute__((aligned(16))) char smem[4 * VIMG];

  const int hkv = blockIdx.x, b = blockIdx.y, split = blockIdx.z, nsplit = gridDim.z;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int qi = lane & 15, grp = lane >> 4;

  const int S_b = p.seq_lens ? p.seq_lens[b] : p.S;
  const int chunk = (((S_b + nsplit - 1) / nsplit) + 63) & ~63;
  const int k_begin = split * chunk;
  const int k_end = min(S_b, k_begin + chunk);
  const int nblk = k_end > k_begin ? (k_end - k_begin + KB - 1) / KB : 0;

  // Q^T as the B operand: lane (q, g) holds Q[q][32c + 8g .. +7] for the four 32-d chunks c; q >= G -> 0
  const int hq = hkv * G + qi;
  V8 qf[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    if (qi < G) {
      qf[c] = *reinterpret_cast<const V8*>(static_cast<const T*>(p.q) + b * p.q_sb + hq * p.q_sh + 32 * c + 8 * grp);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) qf[c][j] = (T)0.f;
    }
  }
  const bool en = qi < G && p.bias != nullptr && p.enable != nullptr && p.enable[b * p.en_sb + hq] != 0;
  const bool en_any = __builtin_amdgcn_ballot_w64(en) != 0;

  // K / V rows through buffer descriptors bounded at k_end: rows past it read as zeros (no stale cache rows)
  const T* kbase = static_cast<const T*>(p.k) + b * p.k_sb + hkv * p.k_sh;
  const T* vbase = static_cast<const T*>(p.v) + b * p.v_sb + hkv * p.v_sh;
  const int rows = max(k_end, 1);
  const auto ksrd = __builtin_amdgcn_make_buffer_rsrc((void*)kbase, (short)0, (int)((rows - 1) * p.k_st * 2 + D * 2),
                                                      0x00020000);
  const auto vsrd = __builtin_amdgcn_make_buffer_rsrc((void*)vbase, (short)0, (int)((rows - 1) * p.v_st * 2 + D * 2),
                                                      0x00020000);
  const float* brow = p.bias ? p.bias + b * p.bias_sb : nullptr;
  const auto bsrd = __builtin_amdgcn_make_buffer_rsrc((void*)brow, (short)0, en_any ? p.W * 4 : 0, 0x00020000);
  // the shared opening's rows from batch row 0 (same bits as this row's copy; every row's workgroups read one copy)
  const int shared = min(p.shared, k_end) & ~(KB - 1);
  const T* kbase0 = static_cast<const T*>(p.k) + hkv * p.k_sh;
  const T* vbase0 = static_cast<const T*>(p.v) + hkv * p.v_sh;
  const auto ksrd0 = __builtin_amdgcn_make_buffer_rsrc((void*)kbase0, (short)0,
                                                       (int)(max(shared - 1, 0) * p.k_st * 2 + D * 2), 0x00020000);
  const auto vsrd0 = __builtin_amdgcn_make_buffer_rsrc((void*)vbase0, (short)0,
                                                       (int)(max(shared - 1, 0) * p.v_st * 2 + D * 2), 0x00020000);

  // per-lane constant offsets
  uint32_t koff[2][4];   // K: row (16 hh + q), bytes 64 c + 16 g
#pragma unroll
  for (int hh = 0; hh < 2; ++hh)
#pragma unroll
    for (int c = 0; c < 4; ++c) koff[hh][c] = (uint32_t)((16 * hh + qi) * p.k_st * 2 + 64 * c + 16 * grp);
  const uint32_t vrow_off = (uint32_t)(grp * p.v_st * 2 + 16 * qi);   // V: rows 4 i + g, 16-B piece q
  char* vimg = smem + wave * VIMG;
  // ds_read_b64_tr_b16 base: lane 4 r + c4 of its 16-lane group supplies row 4 g + r, columns 4 c4 .. +3
  const uint32_t tr_base = (uint32_t)(uintptr_t)(lds_void*)vimg + (uint32_t)((4 * grp + (qi >> 2)) * VSTR + (qi & 3) * 8);

  using BV = __attribute__((ext_vector_type(4))) unsigned;
  BV kn[2][4], vn[8];
  f32x4 bn[2];
  auto load_block = [&](int blk) {
    const int key0 = k_begin + blk * KB;
    const bool sh = key0 + KB <= shared;                 // wave-uniform
    const auto kd = sh ? ksrd0 : ksrd;
    const auto vd = sh ? vsrd0 : vsrd;
#pragma unroll
    for (int hh = 0; hh < 2; ++hh)
#pragma unroll
      for (int c = 0; c < 4; ++c)
        kn[hh][c] = __builtin_amdgcn_raw_buffer_load_b128(kd, (int)(koff[hh][c] + key0 * p.k_st * 2), 0, 0);
#pragma unroll
    for (int i = 0; i < 8; ++i)
      vn[i] = __builtin_amdgcn_raw_buffer_load_b128(vd, (int)(vrow_off + (key0 + 4 * i) * p.v_st * 2), 0, 0);
    if (en_any) {
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const BV r = __builtin_amdgcn_raw_buffer_load_b128(bsrd, (key0 + 16 * hh + 4 * grp) * 4, 0, 0);
        bn[hh] = __builtin_bit_cast(f32x4, r);
      }
    }
  };

  float m = kNegInf, l = 0.f;
  f32x4 oacc[8];
#pragma unroll
  for (int db = 0; db < 8; ++db) oacc[db] = f32x4{0.f, 0.f, 0.f, 0.f};

  int blk = wave;
  if (blk < nblk) load_block(blk);
  for (; blk < nblk; blk += 4) {
    const int key0 = k_begin + blk * KB;
    BV kc[2][4];
    f32x4 bc[2];
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      bc[hh] = bn[hh];
#pragma unroll
      for (int c = 0; c < 4; ++c) kc[hh][c] = kn[hh][c];
    }
    // V rows of this block into the wave's LDS image (in-order LDS: the previous block's tr-reads are done)
#pragma unroll
    for (int i = 0; i < 8; ++i) *reinterpret_cast<BV*>(vimg + (4 * i + grp) * VSTR + 16 * qi) = vn[i];
    if (blk + 4 < nblk) load_block(blk + 4);

    // S^T = K . Q^T for the two 16-key halves
    f32x4 sc[2];
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int c = 0; c < 4; ++c) acc = mfma16x32(__builtin_bit_cast(V8, kc[hh][c]), qf[c], acc);
      sc[hh] = acc;
    }
    // scale, credibility bias, length mask (log2 units); block max over this q's 32 keys (4 lanes x 8)
    float mx = kNegInf;
#pragma unroll
    for (int hh = 0; hh < 2; ++hh)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float s = sc[hh][i] * p.scale_log2;
        if (en) s = __builtin_fmaf(bc[hh][i], kLog2e, s);
        s = (key0 + 16 * hh + 4 * grp + i < k_end) ? s : kNegInf;
        sc[hh][i] = s;
        mx = fmaxf(mx, s);
      }
    mx = quad_max16(mx);
    const float mnew = fmaxf(m, mx);
    const float muse = (mnew == kNegInf) ? 0.f : mnew;
    const float alpha = fast_exp2(m - muse);
    float rs = 0.f;
    V8 pb;
#pragma unroll
    for (int hh = 0; hh < 2; ++hh)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float pe = fast_exp2(sc[hh][i] - muse);
        rs += pe;
        pb[4 * hh + i] = (T)pe;
      }
    l = l * alpha + rs;
    m = mnew;
    if (__builtin_amdgcn_ballot_w64(alpha != 1.f)) {
#pragma unroll
      for (int db = 0; db < 8; ++db) oacc[db] *= alpha;
    }
    // O^T += V^T . P^T: per 16-d block two transposed reads (keys 4g..4g+3 and 16+4g..16+4g+3)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the V image writes above have landed
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int db = 0; db < 8; ++db) {
      i16x4 r0, r1;
      asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r0) : "v"(tr_base), "i"(db * 32));
      asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r1) : "v"(tr_base), "i"(16 * VSTR + db * 32));
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      const V8 va = __builtin_bit_cast(V8, __builtin_shufflevector(r0, r1, 0, 1, 2, 3, 4, 5, 6, 7));
      oacc[db] = mfma16x32(va, pb, oacc[db]);
    }
  }

  // row sums: the 4 lanes of a query head hold disjoint keys under the same running max
  l = quad_sum16(l);
  __syncthreads();                                   // every wave is done with its V image: reuse the LDS
  float* red_o = reinterpret_cast<float*>(smem);     // [4 waves][G][D]
  float* red_ml = red_o + 4 * G * D;                 // [4 waves][G][2]
  if (qi < G) {
#pragma unroll
    for (int db = 0; db < 8; ++db)
#pragma unroll
      for (int i = 0; i < 4; ++i) red_o[(wave * G + qi) * D + 16 * db + 4 * grp + i] = oacc[db][i];
    if (grp == 0) {
      red_ml[(wave * G + qi) * 2 + 0] = m;
      red_ml[(wave * G + qi) * 2 + 1] = l;
    }
  }
  __syncthreads();
  for (int idx = tid; idx < G * D; idx += 256) {
    const int g = idx / D, dd = idx % D;
    float M = kNegInf;
#pragma unroll
    for (int w = 0; w < 4; ++w) M = fmaxf(M, red_ml[(w * G + g) * 2]);
    const float Muse = (M == kNegInf) ? 0.f : M;
    float L = 0.f, O = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const float a = fast_exp2(red_ml[(w * G + g) * 2] - Muse);
      L += red_ml[(w * G + g) * 2 + 1] * a;
      O += red_o[(w * G + g) * D + dd] * a;
    }
    const int h = hkv * G + g;
    if (nsplit == 1) {
      static_cast<T*>(p.o)[b * p.o_sb + h * p.o_sh + dd] = (T)(L > 0.f ? O / L : 0.f);
    } else {
      const int64_t slot = ((int64_t)(b * p.Hq + h) * nsplit + split);
      p.ws_o[slot * D + dd] = O;
      if (dd == 0) { p.ws_ml[slot * 2 + 0] = M; p.ws_ml[slot * 2 + 1] = L; }
    }
  }
}

template <typename T, int D>
__global__ __launch_bounds__(D) void decode_combine_kernel(DecodeParams p, int nsplit) {
  const int hq = blockIdx.x, b = blockIdx.y, dd = threadIdx.x;
  const int64_t slot0 = (int64_t)(b * p.Hq + hq) * nsplit;
  float M = kNegInf;
  for (int s = 0; s < nsplit; ++s) M = fmaxf(M, p.ws_ml[(slot0 + s) * 2]);
  const float Muse = (M == kNegInf) ? 0.f : M;
  float L = 0.f, O = 0.f;
  for (int s = 0; s < nsplit; ++s) {
    const float a = fast_exp2(p.ws_ml[(slot0 + s) * 2] - Muse);
    L += p.ws_ml[(slot0 + s) * 2 + 1] * a;
    O += p.ws_o[(slot0 + s) * D + dd] * a;
  }
  static_cast<T*>(p.o)[b * p.o_sb + hq * p.o_sh + dd] = (T)(L > 0.f ? O / L : 0.f);
}

// --------------------------------------------------------------------------------------------
// answer-token logits
// --------------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void answer_logits_kernel(const T* h, int64_t h_rs, const T* w, int64_t w_rs,
                                                            const int32_t* ids, int n, int D, int round_logits,
                                                            float* out) {
  using V8 = typename Vec<T>::x8;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= n) return;
  const T* hr = h + row * h_rs;
  const T* wr = w + (int64_t)ids[row] * w_rs;
  float acc = 0.f;
  for (int d0 = lane * 8; d0 < D; d0 += 512) {
    const V8 a = *reinterpret_cast<const V8*>(hr + d0);
    const V8 c = *reinterpret_cast<const V8*>(wr + d0);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += (float)a[j] * (float)c[j];
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) acc += __shfl_xor(acc, off, 64);
  if (lane == 0) out[row] = round_logits ? (float)(T)acc : acc;
}

// --------------------------------------------------------------------------------------------
// host helpers
// --------------------------------------------------------------------------------------------
// Process-wide kernel selection knobs (cram_set_knob): -1 = automatic.  The environment is read ONCE, at the
// first query, as the initial value (CRAM_PREFILL_VARIANT = 3 | 8, CRAM_DECODE_U = 1 | 2 | 4); launches never
// call getenv.  A knob changed after a hipGraph capture does not alter the captured launches.
// Thread-safe: the environment is read under std::call_once and the values are atomics (a knob set from one
// thread is seen by launches from any other; set knobs before launches whose choice they should affect).
std::atomic<int> g_knob[CRAM_KNOB_COUNT];
std::once_flag g_knob_once;
inline void knobs_init() {
  std::call_once(g_knob_once, [] {
    const char* e = getenv("CRAM_PREFILL_VARIANT");
    g_knob[CRAM_KNOB_PREFILL_VARIANT].store(
        (e && (e[0] == '0' || e[0] == '3' || e[0] == '4' || e[0] == '7' || e[0] == '8')) ? e[0] - '0'
                                                                                                  : -1);
    const char* eu = getenv("CRAM_DECODE_U");
    g_knob[CRAM_KNOB_DECODE_U].store((eu && (eu[0] == '1' || eu[0] == '2' || eu[0] == '4')) ? eu[0] - '0' : -1);
    const char* em = getenv("CRAM_DECODE_MFMA");
    g_knob[CRAM_KNOB_DECODE_MFMA].store((em && (em[0] == '0' || em[0] == '1')) ? em[0] - '0' : -1);
    const char* eg = getenv("CRAM_GEMM_VARIANT");
    g_knob[CRAM_KNOB_GEMM_VARIANT].store((eg && eg[0] >= '0' && eg[0] <= '2') ? eg[0] - '0' : -1);
  });
}
inline int knob(int k) {
  knobs_init();
  return g_knob[k].load(std::memory_order_relaxed);
}

inline bool al16(const void* ptr) { return (reinterpret_cast<uintptr_t>(ptr) & 15u) == 0; }
inline bool m8(int64_t s) { return (s & 7) == 0; }

template <typename T, int D>
int launch_prefill(PrefillParams& p, hipStream_t stream) {
  const int G = p.Hq / p.Hkv;
  p.hp = (G % 4 == 0) ? 4 : (G % 2 == 0) ? 2 : 1;
  // variant 3 (opt-in, knob CRAM_KNOB_PREFILL_VARIANT / env CRAM_PREFILL_VARIANT=3): 32-key tiles, 162 VGPRs -> three waves per SIMD; +4 % at the sweep
  // shape, but on the tiny Qwen2 model its IE noise doubled on one question and broke the parity bar
  // (tools/ie_noise_probe.py), so 64-key tiles at two waves per SIMD stay the default.
  // variant 8: 8-wave workgroups (one per CU), every K/V tile feeds twice the query rows.
  // variant 7: for GQA groups of 7 (Qwen2-7B), 7-wave workgroups = the 7 query heads of one kv head over the same 32
  // rows (hp = 7: every K/V tile feeds all seven heads, and all waves of a block finish together; otherwise hp = 1,
  // 4 row groups of one head).  Automatic for sequences <= 2048: at the Qwen2 layout, B = 33 x T = 962 ran 601 vs
  // 544 TFLOP/s, but B = 1 x T = 8300 582 vs 807 (one 7-wave workgroup per CU instead of two 4-wave ones;
  // tools/ab_prefill_inproc.py, profiles/r02/ab_prefill_hp7.log).  Knob 0 forces the 4-wave layout.
  const int kv = knob(CRAM_KNOB_PREFILL_VARIANT);
  // variant 4: prefill_x32_kernel (two workgroups per CU, 32 rows per wave, hand-ordered MFMA / softmax stream; bf16,
  // d = 128, GQA groups of 4k).  Automatic from 256 query rows: 1.10-1.12x the 4-wave kernel at the IE-sweep shapes,
  // 1.10x / 1.16x at 8.3k tokens unbiased / biased (1.08x round 2's one-wave-per-SIMD x64 kernel, removed in round 4),
  // 1.06x at B = 3 x 517 biased; 0.94x on a B = 2 x 77 call (tools/ab_x32.hip, profiles/r03/x32/)
  if constexpr (D == 128 && std::is_same<T, __bf16>::value) {
    if ((kv == 4 || (kv == -1 && p.Tq >= 256)) && G % 4 == 0) {
      p.hp = 4;
      p.nqb = (p.Tq + 31) / 32;
      const int64_t nb = (int64_t)p.nqb * (p.Hq / 4) * p.B;
      if (nb > 0x7fffffff) return CRAM_ERR_INVALID_ARG;
      p.nblocks = (int)nb;
      hipLaunchKernelGGL(prefill_x32_kernel, dim3(p.nblocks), dim3(256), 0, stream, p);
      return hipGetLastError() == hipSuccess ? CRAM_OK : CRAM_ERR_LAUNCH;
    }
  }
  int var = (D == 128 && (kv == 3 || kv == 8)) ? kv : 0;
  if (D == 128 && G % 7 == 0 && (kv == 7 || (kv == -1 && p.Tq <= 2048))) {
    var = 7;
    p.hp = 7;
  }
  const int nw = var == 8 ? 8 : var == 7 ? 7 : 4;
  const int bq = 32 * (nw / p.hp);
  p.nqb = (p.Tq + bq - 1) / bq;
  const int64_t nblocks = (int64_t)p.nqb * (p.Hq / p.hp) * p.B;
  if (nblocks > 0x7fffffff) return CRAM_ERR_INVALID_ARG;
  p.nblocks = (int)nblocks;
  if (var == 3)
    hipLaunchKernelGGL((prefill_kernel<T, D, 32, 3>), dim3(p.nblocks), dim3(256), 0, stream, p);
  else if (var == 8)
    hipLaunchKernelGGL((prefill_kernel<T, D, 64, 1, 8>), dim3(p.nblocks), dim3(512), 0, stream, p);
  else if (var == 7)
    hipLaunchKernelGGL((prefill_kernel<T, D, 64, 1, 7>), dim3(p.nblocks), dim3(448), 0, stream, p);
  else
    hipLaunchKernelGGL((prefill_kernel<T, D, 64, 2>), dim3(p.nblocks), dim3(256), 0, stream, p);
  return hipGetLastError() == hipSuccess ? CRAM_OK : CRAM_ERR_LAUNCH;
}

int dispatch_prefill(PrefillParams& p, int d, int dtype, hipStream_t stream) {
  if (dtype == CRAM_DTYPE_BF16)
    return d == 128 ? launch_prefill<__bf16, 128>(p, stream) : launch_prefill<__bf16, 64>(p, stream);
  return d == 128 ? launch_prefill<_Float16, 128>(p, stream) : launch_prefill<_Float16, 64>(p, stream);
}

template <typename T, int D, int G>
int launch_decode_g(DecodeParams& p, int nsplit, hipStream_t stream) {
  // GQA groups of >= 4 heads at d = 128 run on the matrix cores unless the knob says otherwise
  const int km = knob(CRAM_KNOB_DECODE_MFMA);
  if constexpr (D == 128 && G >= 4) {
    if (km != 0) {
      hipLaunchKernelGGL((decode_mfma_kernel<T, G>), dim3(p.Hkv, p.B, nsplit), dim3(256), 0, stream, p);
      if (hipGetLastError() != hipSuccess) return CRAM_ERR_LAUNCH;
      if (nsplit > 1) {
        hipLaunchKernelGGL((decode_combine_kernel<T, D>), dim3(p.Hq, p.B), dim3(D), 0, stream, p, nsplit);
        if (hipGetLastError() != hipSuccess) return CRAM_ERR_LAUNCH;
      }
      return CRAM_OK;
    }
  }
  // keys per lane group per iteration: with >= 1024 workgroups (e.g. the batch-256 decode leg) occupancy is what
  // keeps K/V reads in flight: U = 1 (114 VGPRs, four waves per SIMD) read 4.73 TB/s, U = 2 (149, three) 4.56,
  // U = 4 (205, two) 4.12 (tools/ab_decode_u.py, B = 256); at 512 workgroups U = 4's deeper per-wave prefetch
  // wins (4.32 vs 4.01 for U = 1).  The knob CRAM_KNOB_DECODE_U = 1 | 2 | 4 overrides (A/B, tests)
  // (G <= 4 only: the G = 7 Qwen2 body does 7/4 the VALU work per byte and ran 2.40 vs 2.96 TB/s with U = 1)
  int u = (G <= 4 && (int64_t)p.Hkv * p.B * nsplit >= 1024) ? 1 : 4;
  const int ku = knob(CRAM_KNOB_DECODE_U);
  if (ku == 1 || ku == 2 || ku == 4) u = ku;
  if (u == 1)
    hipLaunchKernelGGL((decode_kernel<T, D, G, 1>), dim3(p.Hkv, p.B, nsplit), dim3(256), 0, stream, p);
  else if (u == 2)
    hipLaunchKernelGGL((decode_kernel<T, D, G, 2>), dim3(p.Hkv, p.B, nsplit), dim3(256), 0, stream, p);
  else
    hipLaunchKernelGGL((decode_kernel<T, D, G>), dim3(p.Hkv, p.B, nsplit), dim3(256), 0, stream, p);
  if (hipGetLastError() != hipSuccess) return CRAM_ERR_LAUNCH;
  if (nsplit > 1) {
    hipLaunchKernelGGL((decode_combine_kernel<T, D>), dim3(p.Hq, p.B), dim3(D), 0, stream, p, nsplit);
    if (hipGetLastError() != hipSuccess) return CRAM_ERR_LAUNCH;
  }
  return CRAM_OK;
}

template <typename T, int D>
int launch_decode(DecodeParams& p, int G, int nsplit, hipStream_t stream) {
  switch (G) {
    case 1: return launch_decode_g<T, D, 1>(p, nsplit, stream);
    case 2: return launch_decode_g<T, D, 2>(p, nsplit, stream);
    case 4: return launch_decode_g<T, D, 4>(p, nsplit, stream);
    case 7: return launch_decode_g<T, D, 7>(p, nsplit, stream);
    case 8: return launch_decode_g<T, D, 8>(p, nsplit, stream);
    default: return CRAM_ERR_UNSUPPORTED;
  }
}

inline bool dtype_ok(int dtype) { return dtype == CRAM_DTYPE_BF16 || dtype == CRAM_DTYPE_F16; }

}  // namespace

extern "C" {

const char* cram_strerror(int code) {
  switch (code) {
    case CRAM_OK: return "ok";
    case CRAM_ERR_INVALID_ARG: return "invalid argument";
    case CRAM_ERR_UNSUPPORTED: return "unsupported head dim, GQA group size or element type";
    case CRAM_ERR_ALIGNMENT: return "stride not a multiple of 8 elements or pointer not 16-byte aligned";
    case CRAM_ERR_LAUNCH: return "kernel launch failed";
    case CRAM_ERR_WORKSPACE: return "split-S workspace missing or too small";
    default: return "unknown error";
  }
}

int cram_abi_version(void) { return CRAM_ABI_VERSION; }

int cram_set_knob(int which, int value) {
  if (which < 0 || which >= CRAM_KNOB_COUNT) return CRAM_ERR_INVALID_ARG;
  knobs_init();
  if (which == CRAM_KNOB_PREFILL_VARIANT && value != -1 && value != 0 && value != 3 && value != 4 && value != 7 &&
      value != 8)
    return CRAM_ERR_INVALID_ARG;
  if (which == CRAM_KNOB_DECODE_U && value != -1 && value != 1 && value != 2 && value != 4)
    return CRAM_ERR_INVALID_ARG;
  if (which == CRAM_KNOB_DECODE_MFMA && value != -1 && value != 0 && value != 1) return CRAM_ERR_INVALID_ARG;
  if (which == CRAM_KNOB_GEMM_VARIANT && (value < -1 || value > 2)) return CRAM_ERR_INVALID_ARG;
  g_knob[which].store(value);
  return CRAM_OK;
}

int cram_get_knob(int which, int* value) {
  if (which < 0 || which >= CRAM_KNOB_COUNT || !value) return CRAM_ERR_INVALID_ARG;
  *value = knob(which);
  return CRAM_OK;
}

int cram_attn_prefill(const void* q, int64_t q_sb, int64_t q_sh, int64_t q_st, const void* k, int64_t k_sb,
                      int64_t k_sh, int64_t k_st, const void* v, int64_t v_sb, int64_t v_sh, int64_t v_st, void* o,
                      int64_t o_sb, int64_t o_sh, int64_t o_st, int B, int Hq, int Hkv, int Tq, int S, int d,
                      int q_pos0, float scale, const float* bias, int64_t bias_sb, const uint8_t* enable,
                      int64_t en_sb, int W, int dtype, cram_stream_t stream) {
  if (!q || !k || !v || !o) return CRAM_ERR_INVALID_ARG;
  if (B <= 0 || Hq <= 0 || Hkv <= 0 || Tq <= 0 || S <= 0 || Hq % Hkv != 0 || q_pos0 < 0) return CRAM_ERR_INVALID_ARG;
  if ((d != 64 && d != 128) || !dtype_ok(dtype)) return CRAM_ERR_UNSUPPORTED;
  if (!al16(q) || !al16(k) || !al16(v) || !al16(o)) return CRAM_ERR_ALIGNMENT;
  if (!m8(q_sb) || !m8(q_sh) || !m8(q_st) || !m8(k_sb) || !m8(k_sh) || !m8(k_st) || !m8(v_sb) || !m8(v_sh) ||
      !m8(v_st) || !m8(o_sb) || !m8(o_sh) || !m8(o_st))
    return CRAM_ERR_ALIGNMENT;
  if (bias && W < 0) return CRAM_ERR_INVALID_ARG;
  // buffer-descriptor extents are 32-bit byte counts
  if ((int64_t)S * (k_st > v_st ? k_st : v_st) * 2 + 2 * d >= (1ll << 31) || (int64_t)W * 4 >= (1ll << 31))
    return CRAM_ERR_UNSUPPORTED;
  PrefillParams p;
  p.q = q; p.q_sb = q_sb; p.q_sh = q_sh; p.q_st = q_st;
  p.k = k; p.k_sb = k_sb; p.k_sh = k_sh; p.k_st = k_st;
  p.v = v; p.v_sb = v_sb; p.v_sh = v_sh; p.v_st = v_st;
  p.o = o; p.o_sb = o_sb; p.o_sh = o_sh; p.o_st = o_st;
  p.bias = (bias && enable) ? bias : nullptr; p.bias_sb = bias_sb;
  p.enable = (bias && enable) ? enable : nullptr; p.en_sb = en_sb;
  p.B = B; p.Hq = Hq; p.Hkv = Hkv; p.Tq = Tq; p.S = S; p.W = bias ? W : 0; p.q_pos0 = q_pos0;
  p.scale_log2 = scale * kLog2e;
  p.cu = nullptr; p.kv_cache = 0;
  return dispatch_prefill(p, d, dtype, (hipStream_t)stream);
}

int cram_attn_prefill_varlen(const void* q, int64_t q_sh, int64_t q_st, const void* k, int64_t k_sh, int64_t k_st,
                             const void* v, int64_t v_sh, int64_t v_st, void* o, int64_t o_sh, int64_t o_st,
                             const int32_t* cu_seqlens, int B, int max_len, int Hq, int Hkv, int d, float scale,
                             const float* bias, int64_t bias_sb, const uint8_t* enable, int64_t en_sb, int W,
                             int dtype, cram_stream_t stream) {
  if (!q || !k || !v || !o || !cu_seqlens) return CRAM_ERR_INVALID_ARG;
  if (B <= 0 || Hq <= 0 || Hkv <= 0 || max_len <= 0 || Hq % Hkv != 0) return CRAM_ERR_INVALID_ARG;
  if ((d != 64 && d != 128) || !dtype_ok(dtype)) return CRAM_ERR_UNSUPPORTED;
  if (!al16(q) || !al16(k) || !al16(v) || !al16(o)) return CRAM_ERR_ALIGNMENT;
  if (!m8(q_sh) || !m8(q_st) || !m8(k_sh) || !m8(k_st) || !m8(v_sh) || !m8(v_st) || !m8(o_sh) || !m8(o_st))
    return CRAM_ERR_ALIGNMENT;
  if (bias && W < 0) return CRAM_ERR_INVALID_ARG;
  if ((int64_t)max_len * (k_st > v_st ? k_st : v_st) * 2 + 2 * d >= (1ll << 31) || (int64_t)W * 4 >= (1ll << 31))
    return CRAM_ERR_UNSUPPORTED;
  PrefillParams p;
  p.q = q; p.q_sb = 0; p.q_sh = q_sh; p.q_st = q_st;
  p.k = k; p.k_sb = 0; p.k_sh = k_sh; p.k_st = k_st;
  p.v = v; p.v_sb = 0; p.v_sh = v_sh; p.v_st = v_st;
  p.o = o; p.o_sb = 0; p.o_sh = o_sh; p.o_st = o_st;
  p.bias = (bias && enable) ? bias : nullptr; p.bias_sb = bias_sb;
  p.enable = (bias && enable) ? enable : nullptr; p.en_sb = en_sb;
  p.B = B; p.Hq = Hq; p.Hkv = Hkv; p.Tq = max_len; p.S = max_len; p.W = bias ? W : 0; p.q_pos0 = 0;
  p.scale_log2 = scale * kLog2e;
  p.cu = cu_seqlens; p.kv_cache = 0;
  return dispatch_prefill(p, d, dtype, (hipStream_t)stream);
}

int cram_attn_prefill_varlen_cached(const void* q, int64_t q_sh, int64_t q_st, const void* k, int64_t k_sb,
                                    int64_t k_sh, int64_t k_st, const void* v, int64_t v_sb, int64_t v_sh,
                                    int64_t v_st, void* o, int64_t o_sh, int64_t o_st, const int32_t* cu_seqlens,
                                    int B, int max_len, int prefix, int Hq, int Hkv, int d, float scale,
                                    const float* bias, int64_t bias_sb, const uint8_t* enable, int64_t en_sb, int W,
                                    int dtype, cram_stream_t stream) {
  if (!q || !k || !v || !o || !cu_seqlens) return CRAM_ERR_INVALID_ARG;
  if (B <= 0 || Hq <= 0 || Hkv <= 0 || max_len <= 0 || prefix < 0 || Hq % Hkv != 0 || k_sb < 0 || v_sb < 0)
    return CRAM_ERR_INVALID_ARG;
  if ((d != 64 && d != 128) || !dtype_ok(dtype)) return CRAM_ERR_UNSUPPORTED;
  if (!al16(q) || !al16(k) || !al16(v) || !al16(o)) return CRAM_ERR_ALIGNMENT;
  if (!m8(q_sh) || !m8(q_st) || !m8(k_sb) || !m8(k_sh) || !m8(k_st) || !m8(v_sb) || !m8(v_sh) || !m8(v_st) ||
      !m8(o_sh) || !m8(o_st))
    return CRAM_ERR_ALIGNMENT;
  if (bias && W < 0) return CRAM_ERR_INVALID_ARG;
  if ((int64_t)(prefix + max_len) * (k_st > v_st ? k_st : v_st) * 2 + 2 * d >= (1ll << 31) ||
      (int64_t)W * 4 >= (1ll << 31))
    return CRAM_ERR_UNSUPPORTED;
  PrefillParams p;
  p.q = q; p.q_sb = 0; p.q_sh = q_sh; p.q_st = q_st;
  p.k = k; p.k_sb = k_sb; p.k_sh = k_sh; p.k_st = k_st;
  p.v = v; p.v_sb = v_sb; p.v_sh = v_sh; p.v_st = v_st;
  p.o = o; p.o_sb = 0; p.o_sh = o_sh; p.o_st = o_st;
  p.bias = (bias && enable) ? bias : nullptr; p.bias_sb = bias_sb;
  p.enable = (bias && enable) ? enable : nullptr; p.en_sb = en_sb;
  p.B = B; p.Hq = Hq; p.Hkv = Hkv; p.Tq = max_len; p.S = prefix + max_len; p.W = bias ? W : 0; p.q_pos0 = prefix;
  p.scale_log2 = scale * kLog2e;
  p.cu = cu_seqlens; p.kv_cache = 1;
  return dispatch_prefill(p, d, dtype, (hipStream_t)stream);
}

size_t cram_attn_decode_workspace_size(int B, int Hq, int d, int num_splits) {
  if (num_splits <= 1 || B <= 0 || Hq <= 0 || d <= 0) return 0;
  return (size_t)B * Hq * num_splits * (size_t)(d + 2) * sizeof(float);
}

int cram_attn_decode(const void* q, int64_t q_sb, int64_t q_sh, const void* k, int64_t k_sb, int64_t k_sh,
                     int64_t k_st, const void* v, int64_t v_sb, int64_t v_sh, int64_t v_st, void* o, int64_t o_sb,
                     int64_t o_sh, int B, int Hq, int Hkv, int S, const int32_t* seq_lens, int d, float scale,
                     const float* bias, int64_t bias_sb, const uint8_t* enable, int64_t en_sb, int W,
                     int num_splits, void* workspace, size_t workspace_bytes, int dtype, cram_stream_t stream) {
  return cram_attn_decode_shared(q, q_sb, q_sh, k, k_sb, k_sh, k_st, v, v_sb, v_sh, v_st, o, o_sb, o_sh, B, Hq, Hkv,
                                 S, seq_lens, d, scale, bias, bias_sb, enable, en_sb, W, 0, num_splits, workspace,
                                 workspace_bytes, dtype, stream);
}

int cram_attn_decode_shared(const void* q, int64_t q_sb, int64_t q_sh, const void* k, int64_t k_sb, int64_t k_sh,
                            int64_t k_st, const void* v, int64_t v_sb, int64_t v_sh, int64_t v_st, void* o,
                            int64_t o_sb, int64_t o_sh, int B, int Hq, int Hkv, int S, const int32_t* seq_lens, int d,
                            float scale, const float* bias, int64_t bias_sb, const uint8_t* enable, int64_t en_sb,
                            int W, int shared_rows, int num_splits, void* workspace, size_t workspace_bytes, int dtype,
                            cram_stream_t stream) {
  if (!q || !k || !v || !o || shared_rows < 0) return CRAM_ERR_INVALID_ARG;
  if (B <= 0 || Hq <= 0 || Hkv <= 0 || S <= 0 || Hq % Hkv != 0 || num_splits <= 0 || B > 65535 ||
      num_splits > 65535)
    return CRAM_ERR_INVALID_ARG;
  if ((d != 64 && d != 128) || !dtype_ok(dtype)) return CRAM_ERR_UNSUPPORTED;
  if (!al16(q) || !al16(k) || !al16(v)) return CRAM_ERR_ALIGNMENT;
  if (!m8(q_sb) || !m8(q_sh) || !m8(k_sb) || !m8(k_sh) || !m8(k_st) || !m8(v_sb) || !m8(v_sh) || !m8(v_st))
    return CRAM_ERR_ALIGNMENT;
  if (bias && W < 0) return CRAM_ERR_INVALID_ARG;
  DecodeParams p;
  p.q = q; p.q_sb = q_sb; p.q_sh = q_sh;
  p.k = k; p.k_sb = k_sb; p.k_sh = k_sh; p.k_st = k_st;
  p.v = v; p.v_sb = v_sb; p.v_sh = v_sh; p.v_st = v_st;
  p.o = o; p.o_sb = o_sb; p.o_sh = o_sh;
  p.bias = (bias && enable) ? bias : nullptr; p.bias_sb = bias_sb;
  p.enable = (bias && enable) ? enable : nullptr; p.en_sb = en_sb;
  p.seq_lens = seq_lens;
  p.B = B; p.Hq = Hq; p.Hkv = Hkv; p.S = S; p.W = bias ? W : 0;
  p.scale_log2 = scale * kLog2e;
  p.ws_o = nullptr; p.ws_ml = nullptr;
  p.shared = shared_rows & ~31;
  if (num_splits > 1) {
    const size_t need = cram_attn_decode_workspace_size(B, Hq, d, num_splits);
    if (!workspace || workspace_bytes < need || !al16(workspace)) return CRAM_ERR_WORKSPACE;
    p.ws_o = (float*)workspace;
    p.ws_ml = p.ws_o + (size_t)B * Hq * num_splits * d;
  }
  const int G = Hq / Hkv;
  const hipStream_t st = (hipStream_t)stream;
  if (dtype == CRAM_DTYPE_BF16)
    return d == 128 ? launch_decode<__bf16, 128>(p, G, num_splits, st) : launch_decode<__bf16, 64>(p, G, num_splits, st);
  return d == 128 ? launch_decode<_Float16, 128>(p, G, num_splits, st)
                  : launch_decode<_Float16, 64>(p, G, num_splits, st);
}

int cram_answer_logits(const void* hidden, int64_t h_rs, const void* w_lm, int64_t w_rs, const int32_t* ids, int n,
                       int D, int round_logits, float* out, int dtype, cram_stream_t stream) {
  if (!hidden || !w_lm || !ids || !out || n < 0 || D <= 0) return CRAM_ERR_INVALID_ARG;
  if (!dtype_ok(dtype)) return CRAM_ERR_UNSUPPORTED;
  if (n == 0) return CRAM_OK;
  if ((D & 7) || !m8(h_rs) || !m8(w_rs) || !al16(hidden) || !al16(w_lm)) return CRAM_ERR_ALIGNMENT;
  const dim3 g((n + 3) / 4);
  const hipStream_t st = (hipStream_t)stream;
  if (dtype == CRAM_DTYPE_BF16)
    hipLaunchKernelGGL(answer_logits_kernel<__bf16>, g, dim3(256), 0, st, (const __bf16*)hidden, h_rs,
                       (const __bf16*)w_lm, w_rs, ids, n, D, round_logits, out);
  else
    hipLaunchKernelGGL(answer_logits_kernel<_Float16>, g, dim3(256), 0, st, (const _Float16*)hidden, h_rs,
                       (const _Float16*)w_lm, w_rs, ids, n, D, round_logits, out);
  return hipGetLastError() == hipSuccess ? CRAM_OK : CRAM_ERR_LAUNCH;
}

}  // extern "C"
