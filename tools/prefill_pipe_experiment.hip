// Experiment (not part of the library): a software-pipelined, one-wave-per-SIMD variant of the credibility-biased
// prefill kernel, kept with its measurement.  Build and run on an MI355X:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/prefill_pipe_experiment.hip -o tools/prefill_pipe_experiment
//   tools/prefill_pipe_experiment            (sweep shape B=33 T=962 and B=1 T=8300, Llama-3 GQA 32/8, d 128)
// Design: 4-stage LDS-DMA ring (K, V and per-head bias rows), counted vmcnt + raw barrier, QK^T of tile t+1 in one
// basic block with the exponentials of tile t and PV of tile t, V^T reads by inline asm with a dependency-carrying
// lgkmcnt wait.  Result (ROCm 7.2 hipcc, round 1): correct (same parity suite as the library kernel while it was
// wired in), but 0.67-0.73x the library kernel's throughput: the ~350-register live set makes hipcc place the MFMA
// accumulators (S and O) in AGPRs, and the softmax (S) and O rescale then cost ~160 v_accvgpr moves per tile.
// Making it pay needs explicit register ownership (hand-written asm: S in arch VGPRs, O and Q in AGPRs).
#include "../cram_amd/csrc/cram_attn.hip"

#include <cstdio>
#include <random>
#include <type_traits>
#include <vector>

namespace {
// lgkmcnt(0) that carries the tr-read results as in/out operands: the MFMAs consuming them cannot be scheduled
// above the wait, and nothing else is fenced (no sched_barrier)
__device__ __forceinline__ void lgkm0_dep(i16x4 (&rr)[16]) {
  asm volatile("s_waitcnt lgkmcnt(0)"
               : "+v"(rr[0]), "+v"(rr[1]), "+v"(rr[2]), "+v"(rr[3]), "+v"(rr[4]), "+v"(rr[5]), "+v"(rr[6]),
                 "+v"(rr[7]), "+v"(rr[8]), "+v"(rr[9]), "+v"(rr[10]), "+v"(rr[11]), "+v"(rr[12]), "+v"(rr[13]),
                 "+v"(rr[14]), "+v"(rr[15]));
}
template <typename T, int VSTR, int KB>
__device__ __forceinline__ void pv_block32_dep(uint32_t vaddr, const f32x16& pk, f32x16 (&oacc)[4]) {
  using V8 = typename Vec<T>::x8;
  V8 pb[2];
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
    for (int j = 0; j < 8; ++j) pb[s2][j] = (T)pk[8 * s2 + j];
  i16x4 rr[16];
  tr_reads32<VSTR, KB>(vaddr, rr);
  lgkm0_dep(rr);
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
    for (int db = 0; db < 4; ++db)
      oacc[db] = mfma32x16(__builtin_bit_cast(V8, __builtin_shufflevector(rr[8 * s2 + 2 * db], rr[8 * s2 + 2 * db + 1],
                                                                          0, 1, 2, 3, 4, 5, 6, 7)), pb[s2], oacc[db]);
}

// --------------------------------------------------------------------------------------------
// prefill, software-pipelined: one wave per SIMD
// --------------------------------------------------------------------------------------------
// Same LDS images, staging and score arithmetic as prefill_kernel, restructured for ONE workgroup per CU so each
// wave owns a SIMD (and its 512-register file) and keeps the matrix pipe fed by itself:
//   step t   A.  S(t+1) = K(t+1).Q^T  (16 MFMAs)  in one basic block with the row max + exponentials of S(t)
//            B.  O = alpha.O + V(t)^T.P(t)^T  (16 MFMAs) beside the row sums; the LDS-DMA of tile t+3 issued
// K/V tiles live in a 4-stage LDS ring (tile t+3 lands while t+2 waits and t+1 / t are read); one raw barrier per
// tile behind a counted vmcnt that leaves tile t+3's DMA in flight.  The two score tiles alternate between two
// register sets (the loop is unrolled by two so the roles are static).
// A workgroup = hp query heads of one kv head x 32*(4/hp) rows; the rows are STRIDED over the waves of a head
// (row = q0 + rw*lane + wave/hp), so every wave spans the block's whole causal range and all waves run the same
// tiles (hp = 4: Llama-3 GQA 4:1, rows contiguous; hp = 1: MHA or GQA 7:1).

// max of 32 scores as a tree: an exact max does not depend on the order, a serial chain's latency does
__device__ __forceinline__ float max32(const f32x16& a, const f32x16& b) {
  float x[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) x[i] = fmaxf(fmaxf(a[2 * i], a[2 * i + 1]), fmaxf(b[2 * i], b[2 * i + 1]));
#pragma unroll
  for (int i = 0; i < 4; ++i) x[i] = fmaxf(x[i], x[i + 4]);
  return fmaxf(fmaxf(x[0], x[2]), fmaxf(x[1], x[3]));
}

template <typename T, int D>
__global__ __launch_bounds__(256, 1) void prefill_pipe_kernel(PrefillParams p) {
  using C = PrefillCfg<D, 64>;
  using V8 = typename Vec<T>::x8;
  using V4 = typename Vec<T>::x4;
  constexpr int NS = 4;                                   // ring stages (power of two)
  constexpr int KCH = C::KCH, NCH = C::KCH + C::VCH;
  constexpr int CPW = (NCH + 3) / 4;
  static_assert(C::NKB == 2 && (NS & (NS - 1)) == 0, "64-key tiles, power-of-two ring");
  static_assert(CPW + 1 <= 15, "vmcnt immediates below");
  // a stage = the padded K | V images of prefill_kernel + one 64-key bias row PER WAVE (its head's: staged only
  // for an enabled head, zeros otherwise, so the exponent formula below needs no per-head branch)
  constexpr int STG = C::B_OFF + 4 * C::B_BYTES;
  __shared__ __attribute__((aligned(16))) char smem[NS * STG];

  const int bid = blockIdx.x;
  const int xcd = bid & 7, q8 = p.nblocks >> 3, r8 = p.nblocks & 7;
  const int wid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int hp = p.hp, rw = 4 / hp, BQ = 32 * rw;
  const int nhg = p.Hq / hp;
  const int qi_blk = wid % p.nqb;
  const int bh = wid / p.nqb;
  const int hg = bh % nhg;
  const int b = bh / nhg;
  const int qblk = p.nqb - 1 - qi_blk;          // heaviest (longest causal range) first
  const int G = p.Hq / p.Hkv;
  const int hkv = (hg * hp) / G;

  int Tq = p.Tq, S = p.S, q_pos0 = p.q_pos0;
  int64_t tok0 = 0;
  if (p.cu) {
    tok0 = p.cu[b];
    Tq = S = p.cu[b + 1] - (int)tok0;
    q_pos0 = 0;
    if (qblk * BQ >= Tq) return;               // whole workgroup exits before any barrier
  }
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, hh = lane >> 5;
  const int hq = hg * hp + wave % hp;
  const int rsub = wave / hp;                   // this wave's row phase in the block
  const int q_row0 = qblk * BQ;
  const int qrow = q_row0 + rw * r + rsub;
  const int qpos = q_pos0 + qrow;

  const T* qb = static_cast<const T*>(p.q) + b * p.q_sb + tok0 * p.q_st + hq * p.q_sh;
  const T* kbase = static_cast<const T*>(p.k) + b * p.k_sb + tok0 * p.k_st + hkv * p.k_sh;
  const T* vbase = static_cast<const T*>(p.v) + b * p.v_sb + tok0 * p.v_st + hkv * p.v_sh;
  const bool has_bias = (p.bias != nullptr) && (p.enable != nullptr);
  const bool en = has_bias && p.enable[b * p.en_sb + hq] != 0;
  const float* brow = en ? p.bias + b * p.bias_sb : nullptr;

  V8 qf[D / 16];
#pragma unroll
  for (int ks = 0; ks < D / 16; ++ks) {
    if (qrow < Tq) {
      qf[ks] = *reinterpret_cast<const V8*>(qb + qrow * p.q_st + 16 * ks + 8 * hh);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) qf[ks][j] = (T)0.f;
    }
  }

  const int blk_last_q = min(q_row0 + BQ, Tq) - 1;
  const int kv_end = min(S, q_pos0 + blk_last_q + 1);
  const int nt = (kv_end + C::BK - 1) / C::BK;   // >= 1: the block's first row sees key 0
  const int wave_qpos_min = q_pos0 + q_row0 + rsub;
  const int wave_qpos_max = q_pos0 + min(q_row0 + rw * 31 + rsub, Tq - 1);

  // LDS-DMA staging exactly as prefill_kernel (chunk c of a tile's padded K | V image is fetched by wave c % 4)
  uint32_t doff[CPW];
#pragma unroll
  for (int i = 0; i < CPW; ++i) {
    const int c = wave + 4 * i;
    uint32_t off = 0xFFFFFFF0u;
    if (c < KCH) {
      const int x = c * 1024 + 16 * lane, row = x / C::KSTR, colb = x % C::KSTR;
      if (x < C::K_BYTES && colb < D * 2) off = (uint32_t)(row * p.k_st * 2 + colb);
    } else if (c < NCH) {
      const int x = (c - KCH) * 1024 + 16 * lane, row = x / C::VSTR, colb = x % C::VSTR;
      if (x < C::V_BYTES && colb < D * 2) off = (uint32_t)(row * p.v_st * 2 + colb);
    }
    doff[i] = off;
  }
  auto gload = [&](int t) {                    // K/V of tile t -> ring stage t % NS (asynchronous)
    const int key0 = t * C::BK;
    const int rows_left = S - key0;
    const auto ksrd = __builtin_amdgcn_make_buffer_rsrc((void*)(kbase + (int64_t)key0 * p.k_st), (short)0,
                                                        (int)((rows_left - 1) * p.k_st * 2 + D * 2), 0x00020000);
    const auto vsrd = __builtin_amdgcn_make_buffer_rsrc((void*)(vbase + (int64_t)key0 * p.v_st), (short)0,
                                                        (int)((rows_left - 1) * p.v_st * 2 + D * 2), 0x00020000);
    char* base = smem + (t & (NS - 1)) * STG;
#pragma unroll
    for (int i = 0; i < CPW; ++i) {
      const int c = wave + 4 * i;
      if (c < KCH)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(ksrd, (lds_void*)(base + c * 1024), 16, (int)doff[i], 0, 0, 0);
      else if (c < NCH)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(vsrd, (lds_void*)(base + c * 1024), 16, (int)doff[i], 0, 0, 0);
    }
    // the tile's bias row (natural-log units) for this wave's head if it is enabled: 64 lanes x 4 B into the
    // wave's own row of the stage; keys >= W read as 0
    if (en) {
      const int wl = p.W - key0;
      const auto bsrd = __builtin_amdgcn_make_buffer_rsrc((void*)(brow + key0), (short)0, wl > 0 ? wl * 4 : 0,
                                                          0x00020000);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(bsrd, (lds_void*)(base + C::B_OFF + wave * C::B_BYTES), 4, lane * 4,
                                               0, 0, 0);
    }
  };
  // vmcnt <= (this wave's DMA pieces of the newest tile): retires the older tiles' pieces.
  // gfx9 s_waitcnt encoding: vmcnt[3:0], expcnt 7, lgkmcnt 15.
  auto wait_older_tiles = [&]() {
    if (en) {                                  // + the bias piece
      if (wave == 0) __builtin_amdgcn_s_waitcnt(0x0F70 | ((NCH + 3) / 4 + 1));
      else if (wave == 1) __builtin_amdgcn_s_waitcnt(0x0F70 | ((NCH + 2) / 4 + 1));
      else if (wave == 2) __builtin_amdgcn_s_waitcnt(0x0F70 | ((NCH + 1) / 4 + 1));
      else __builtin_amdgcn_s_waitcnt(0x0F70 | (NCH / 4 + 1));
    } else {
      if (wave == 0) __builtin_amdgcn_s_waitcnt(0x0F70 | ((NCH + 3) / 4));
      else if (wave == 1) __builtin_amdgcn_s_waitcnt(0x0F70 | ((NCH + 2) / 4));
      else if (wave == 2) __builtin_amdgcn_s_waitcnt(0x0F70 | ((NCH + 1) / 4));
      else __builtin_amdgcn_s_waitcnt(0x0F70 | (NCH / 4));
    }
  };
  // raw barrier behind lgkmcnt(0) (this wave's LDS writes): a __syncthreads() would also drain vmcnt, i.e. the
  // DMA kept in flight
  auto barrier = [&]() {
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_barrier();
  };

  float m = kNegInf, l = 0.f;
  f32x16 oacc[D / 32];
#pragma unroll
  for (int db = 0; db < D / 32; ++db)
#pragma unroll
    for (int e = 0; e < 16; ++e) oacc[db][e] = 0.f;
  const f32x16 zero16 = {};
  const int g16 = lane >> 4, i16 = lane & 15;
  const int tr_key = 4 * (g16 >> 1) + (i16 >> 2);
  const int tr_col = 16 * (g16 & 1) + 4 * (i16 & 3);

  auto qk = [&](int t, f32x16 (&s)[2]) {       // S^T(t) = K(t).Q^T
    const char* base = smem + (t & (NS - 1)) * STG;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int ks = 0; ks < D / 16; ++ks) {
        const V8 a = *reinterpret_cast<const V8*>(base + (kb * 32 + r) * C::KSTR + (16 * ks + 8 * hh) * 2);
        s[kb] = mfma32x16(a, qf[ks], ks == 0 ? zero16 : s[kb]);
      }
  };
  const uint32_t tr_lane = (uint32_t)(tr_key * C::VSTR + tr_col * 2);
  static_assert(D == 128, "pv_block32 covers four 32-column blocks");

  // order of phase A in the scheduler: 4 K-fragment reads ahead, then each MFMA with the next read and 5 VALU
  // (keeps ~4 fragments = 16 VGPRs in flight instead of all 16, and spreads the softmax over the MFMA gaps)
  auto interleave_qk = [&]() {
    __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
#pragma unroll
    for (int i = 0; i < 12; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x402, 5, 0);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x402, 5, 0);
    }
  };

  // one pipeline step: probabilities of S(t) beside QK^T of tile t+1 (if kNext), then PV of tile t
  auto step = [&](int t, f32x16 (&cur)[2], f32x16 (&nxt)[2], auto next_tag) {
    constexpr bool kNext = decltype(next_tag)::value;
    const int key0 = t * C::BK;
    const float* bl = reinterpret_cast<const float*>(smem + (t & (NS - 1)) * STG + C::B_OFF + wave * C::B_BYTES);
    const bool need_mask = (key0 + C::BK - 1 > wave_qpos_min) || (key0 + C::BK > S);
    // ---- A1: row max of tile t in log2 units, max over s*c + b*log2e (b = 0 for a head that is not enabled)
    float mx;
    if (!need_mask && !en) {                   // plain: max of the raw scores, scaled once (fl(c*s) is monotone)
      mx = max32(cur[0], cur[1]) * p.scale_log2;
    } else if (!need_mask) {                   // biased interior tile
      float mp[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int kb = i >> 2, g = i & 3;
        const f32x4 bv = *reinterpret_cast<const f32x4*>(bl + kb * 32 + 8 * g + 4 * hh);
        mp[i] = fmaxf(fmaxf(__builtin_fmaf(cur[kb][4 * g], p.scale_log2, bv[0] * kLog2e),
                            __builtin_fmaf(cur[kb][4 * g + 1], p.scale_log2, bv[1] * kLog2e)),
                      fmaxf(__builtin_fmaf(cur[kb][4 * g + 2], p.scale_log2, bv[2] * kLog2e),
                            __builtin_fmaf(cur[kb][4 * g + 3], p.scale_log2, bv[3] * kLog2e)));
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) mp[i] = fmaxf(mp[i], mp[i + 4]);
      mx = fmaxf(fmaxf(mp[0], mp[2]), fmaxf(mp[1], mp[3]));
    } else {                                   // diagonal / ragged tile: scaled scores, causal / length mask
      const int lim = min(qpos, S - 1) - key0;
      float mp[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int kb = i >> 2, g = i & 3;
        const f32x4 bv = *reinterpret_cast<const f32x4*>(bl + kb * 32 + 8 * g + 4 * hh);
        float x[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const bool dead = kb * 32 + 8 * g + 4 * hh + e > lim;
          cur[kb][4 * g + e] = dead ? kNegInf : cur[kb][4 * g + e] * p.scale_log2;   // x: bias not yet added
          x[e] = dead ? kNegInf : __builtin_fmaf(cur[kb][4 * g + e], 1.f, bv[e] * kLog2e);
        }
        mp[i] = fmaxf(fmaxf(x[0], x[1]), fmaxf(x[2], x[3]));
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) mp[i] = fmaxf(mp[i], mp[i + 4]);
      mx = fmaxf(fmaxf(mp[0], mp[2]), fmaxf(mp[1], mp[3]));
    }
    const float mnew = fmaxf(m, half_max(mx));
    const float muse = (mnew == kNegInf) ? 0.f : mnew;
    const float alpha = fast_exp2(m - muse);
    m = mnew;
    // ---- A2 + B in ONE basic block (no branches): QK^T of tile t+1, the exponentials of tile t
    //   p = exp2(fma(x, c1, fma(b, log2e, -m)))  with x the raw score and c1 = scale (interior tiles) or x the
    //   scaled, masked score and c1 = 1 (diagonal / ragged tiles); b is the wave's own bias row: 0 for a head
    //   that is not enabled, so fma(0, log2e, -m) = -m and a zero bias stays bit-identical to no bias;
    //   -inf biases and masked keys give -inf exponents, never NaN;
    // the O rescale (unconditional: a branch here would split the block), PV of the tile's first 32 keys, the
    // row sums.  The V^T reads are inline asm with a dependency-carrying wait (pv_block32_dep).
    const float c1 = need_mask ? 1.f : p.scale_log2;
    if constexpr (kNext) qk(t + 1, nxt);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int kb = i >> 2, g = i & 3;
      const f32x4 bv = *reinterpret_cast<const f32x4*>(bl + kb * 32 + 8 * g + 4 * hh);
#pragma unroll
      for (int e = 0; e < 4; ++e)
        cur[kb][4 * g + e] = fast_exp2(__builtin_fmaf(cur[kb][4 * g + e], c1, __builtin_fmaf(bv[e], kLog2e, -muse)));
    }
#pragma unroll
    for (int db = 0; db < D / 32; ++db)
#pragma unroll
      for (int e = 0; e < 16; ++e) oacc[db][e] *= alpha;
    const uint32_t vaddr = (uint32_t)(uintptr_t)(lds_void*)(smem + (t & (NS - 1)) * STG + C::V_OFF) + tr_lane;
    pv_block32_dep<T, C::VSTR, 0>(vaddr, cur[0], oacc);
    float r4[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int e = 0; e < 16; ++e) r4[e & 3] += cur[kb][e];
    l = l * alpha + half_sum((r4[0] + r4[1]) + (r4[2] + r4[3]));
    // the upper 32 keys lie past every row of this wave (diagonal tile): their probabilities are exactly 0
    if (key0 + 32 <= wave_qpos_max) pv_block32_dep<T, C::VSTR, 1>(vaddr, cur[1], oacc);
    // DMA of tile t+3 into the stage tile t-1 used (every wave passed the previous barrier)
    if (t + NS - 1 < nt) gload(t + NS - 1);
    // ---- end of tile: tile t+2 landed (this wave's pieces; the barrier covers the others')
    if (t + NS - 1 < nt) wait_older_tiles();
    else __builtin_amdgcn_s_waitcnt(kWaitVmcnt0);
    barrier();
  };

  // prologue: zero every stage's bias row (read by the exponent formula even when no head is biased), then
  // Q and tiles 0 .. NS-2 resident; S(0)
#pragma unroll
  for (int i = 0; i < NS; ++i)                 // NS stages x 4 rows x 64 floats = 256 threads x NS
    reinterpret_cast<float*>(smem + i * STG + C::B_OFF)[tid] = 0.f;
  __syncthreads();
#pragma unroll
  for (int t = 0; t < NS - 1; ++t)
    if (t < nt) gload(t);
  __builtin_amdgcn_s_waitcnt(kWaitVmcnt0);
  barrier();
  f32x16 sa[2], sb[2];
  qk(0, sa);
  int t = 0;
  for (; t + 2 < nt; t += 2) {
    step(t, sa, sb, std::true_type{});
    step(t + 1, sb, sa, std::true_type{});
  }
  if (t + 1 < nt) {
    step(t, sa, sb, std::true_type{});
    step(t + 1, sb, sa, std::false_type{});
  } else {
    step(t, sa, sb, std::false_type{});
  }

  // every wave passed the last tile's barrier: the ring is free for the O staging rows
  store_o_rows<T, D>(smem + wave * 32 * (D * 2 + 16), oacc, l > 0.f ? 1.f / l : 0.f, r, hh, lane,
                     static_cast<T*>(p.o) + b * p.o_sb + tok0 * p.o_st + hq * p.o_sh, p.o_st, q_row0 + rsub, rw, Tq);
}

}  // namespace

int main() {
  const int shapes[2][2] = {{33, 962}, {1, 8300}};
  for (const auto& sh : shapes) {
    const int B = sh[0], T = sh[1], Hq = 32, Hkv = 8, d = 128;
    const size_t nq = (size_t)B * T * Hq * d, nk = (size_t)B * T * Hkv * d;
    std::vector<__bf16> hq(nq), hk(nk), hv(nk);
    std::mt19937 rng(1);
    std::normal_distribution<float> nd(0.f, 1.f);
    for (auto& x : hq) x = (__bf16)nd(rng);
    for (auto& x : hk) x = (__bf16)nd(rng);
    for (auto& x : hv) x = (__bf16)nd(rng);
    __bf16 *q, *k, *v, *o1, *o2;
    hipMalloc(&q, nq * 2); hipMalloc(&k, nk * 2); hipMalloc(&v, nk * 2); hipMalloc(&o1, nq * 2); hipMalloc(&o2, nq * 2);
    hipMemcpy(q, hq.data(), nq * 2, hipMemcpyHostToDevice);
    hipMemcpy(k, hk.data(), nk * 2, hipMemcpyHostToDevice);
    hipMemcpy(v, hv.data(), nk * 2, hipMemcpyHostToDevice);
    PrefillParams p{};
    p.q = q; p.q_sb = (int64_t)T * Hq * d; p.q_sh = d; p.q_st = (int64_t)Hq * d;
    p.k = k; p.k_sb = (int64_t)Hkv * T * d; p.k_sh = (int64_t)T * d; p.k_st = d;
    p.v = v; p.v_sb = p.k_sb; p.v_sh = p.k_sh; p.v_st = d;
    p.o_sb = p.q_sb; p.o_sh = d; p.o_st = p.q_st;
    p.B = B; p.Hq = Hq; p.Hkv = Hkv; p.Tq = T; p.S = T; p.W = 0; p.q_pos0 = 0;
    p.scale_log2 = kLog2e / sqrtf((float)d);
    p.hp = 4; p.nqb = (T + 31) / 32; p.nblocks = p.nqb * (Hq / 4) * B;
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    float ms[2];
    for (int which = 0; which < 2; ++which) {
      p.o = which ? (void*)o2 : (void*)o1;
      auto run = [&]() {
        if (which) hipLaunchKernelGGL((prefill_pipe_kernel<__bf16, 128>), dim3(p.nblocks), dim3(256), 0, 0, p);
        else hipLaunchKernelGGL((prefill_kernel<__bf16, 128, 64, 2>), dim3(p.nblocks), dim3(256), 0, 0, p);
      };
      for (int i = 0; i < 3; ++i) run();
      hipEventRecord(e0);
      for (int i = 0; i < 20; ++i) run();
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      hipEventElapsedTime(&ms[which], e0, e1);
      ms[which] /= 20;
    }
    std::vector<__bf16> a(nq), c(nq);
    hipMemcpy(a.data(), o1, nq * 2, hipMemcpyDeviceToHost);
    hipMemcpy(c.data(), o2, nq * 2, hipMemcpyDeviceToHost);
    double md = 0;
    for (size_t i = 0; i < nq; ++i) md = fmax(md, fabs((double)(float)a[i] - (double)(float)c[i]));
    const double fl = 4.0 * d * Hq * B * (double)T * (T + 1) / 2;
    printf("B=%d T=%d: library %.3f ms (%.0f TF/s), pipelined %.3f ms (%.0f TF/s), max|diff| %.2e\n", B, T, ms[0],
           fl / ms[0] / 1e9, ms[1], fl / ms[1] / 1e9, md);
    hipFree(q); hipFree(k); hipFree(v); hipFree(o1); hipFree(o2);
  }
  return 0;
}
