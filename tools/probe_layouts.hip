// Hardware probe: MFMA 32x32x16 bf16 C/D layout and ds_read_b64_tr_b16 semantics on gfx950.
// Prints mismatches against the maps the prefill kernel assumes.
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) i16x4 lds_i16x4;

__global__ void mfma_probe(float* out, int mode) {
  int lane = threadIdx.x, r = lane & 31, h = lane >> 5;
  bf16x8 a, b;
  for (int j = 0; j < 8; ++j) {
    int k = 8 * h + j;
    // mode 0: A[i][k] = (k==0) ? i : 0, B[k][n] = (k==0)   -> C[i][n] = i
    // mode 1: A[i][k] = (k==0),          B[k][n] = (k==0) ? n : 0 -> C[i][n] = n
    // mode 2: A[i][k] = (k==i%16)?1:0,   B[k][n] = k          -> C[i][n] = i%16 (k map check)
    float av, bv;
    if (mode == 0) { av = (k == 0) ? r : 0; bv = (k == 0) ? 1 : 0; }
    else if (mode == 1) { av = (k == 0) ? 1 : 0; bv = (k == 0) ? r : 0; }
    else { av = (k == (r % 16)) ? 1 : 0; bv = k; }
    a[j] = (__bf16)av; b[j] = (__bf16)bv;
  }
  f32x16 c = {};
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  for (int e = 0; e < 16; ++e) out[lane * 16 + e] = c[e];
}

__global__ void tr_probe(short* out) {
  __shared__ short tile[16 * 72];  // 16 rows x 64 cols, row stride 72 elements
  for (int i = threadIdx.x; i < 16 * 72; i += 64) tile[i] = (short)((i / 72) * 100 + (i % 72));
  __syncthreads();
  int lane = threadIdx.x, g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  int row = 4 * g + q, col = 4 * p;  // group g reads rows 4g..4g+3, cols 0..15
  i16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(tile + row * 72 + col));
  for (int e = 0; e < 4; ++e) out[lane * 4 + e] = v[e];
}

int main() {
  float* d; short* ds;
  hipMalloc(&d, 64 * 16 * 4);
  hipMalloc(&ds, 64 * 4 * 2);
  float hbuf[64 * 16];
  int bad = 0;
  for (int mode = 0; mode < 3; ++mode) {
    hipLaunchKernelGGL(mfma_probe, dim3(1), dim3(64), 0, 0, d, mode);
    hipMemcpy(hbuf, d, sizeof(hbuf), hipMemcpyDeviceToHost);
    for (int lane = 0; lane < 64; ++lane)
      for (int e = 0; e < 16; ++e) {
        int row = (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5), col = lane & 31;
        float want = mode == 0 ? row : mode == 1 ? col : (row % 16);
        if (hbuf[lane * 16 + e] != want) {
          if (bad < 20) printf("mfma mode %d lane %d reg %d got %g want %g\n", mode, lane, e, hbuf[lane * 16 + e], want);
          ++bad;
        }
      }
  }
  short sb[64 * 4];
  hipLaunchKernelGGL(tr_probe, dim3(1), dim3(64), 0, 0, ds);
  hipMemcpy(sb, ds, sizeof(sb), hipMemcpyDeviceToHost);
  for (int lane = 0; lane < 64; ++lane)
    for (int e = 0; e < 4; ++e) {
      int g = lane >> 4, i = lane & 15;
      short want = (short)((4 * g + e) * 100 + i);
      if (sb[lane * 4 + e] != want) {
        if (bad < 40) printf("tr lane %d elem %d got %d want %d\n", lane, e, sb[lane * 4 + e], want);
        ++bad;
      }
    }
  printf("probe mismatches: %d\n", bad);
  return bad != 0;
}
