// Diagnostic: where gemm_w4_kernel's K-tile time goes.  Builds cram_gemm.hip with -DCRAM_W4_STAMPS (the stamped
// instruction stream of tools/gen_gemm_w4.py, variant S: s_memtime brackets around the three rendezvous of every
// K-tile), runs the gate/up shape (M 29184, N 28672, K 4096, random bf16) and prints the mean shader cycles per K-tile:
// whole tile, B1 (lgkmcnt + barrier after the activation reads), B2 (after the weight reads), B3 (vmcnt + barrier
// before the next tile's reads).  Stamps cost ~40 cycles each; the stream is otherwise the product's.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DCRAM_W4_STAMPS -I include tools/w4_stamps.hip -o tools/w4_stamps
#include "../cram_amd/csrc/cram_gemm.hip"

#include <cstdio>
#include <vector>

extern "C" int cram_get_knob(int, int* v) { *v = 1; return 0; }

__global__ void fill(__bf16* p, size_t n, unsigned seed, float scale) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    unsigned h = (unsigned)i * 2654435761u ^ seed;
    h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
    p[i] = (__bf16)(((h & 0xFFFF) / 32768.0f - 1.0f) * scale);
  }
}

int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 29184, N = argc > 2 ? atoi(argv[2]) : 28672, K = argc > 3 ? atoi(argv[3]) : 4096;
  __bf16 *x, *w, *o;
  hipMalloc(&x, (size_t)M * K * 2); hipMalloc(&w, (size_t)N * K * 2); hipMalloc(&o, (size_t)M * N * 2);
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, x, (size_t)M * K, 1u, 1.0f);
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, w, (size_t)N * K, 2u, 1.0f / 64);
  const int nb = ((M + 255) / 256) * (N / 256);
  unsigned* st;
  hipMalloc(&st, (size_t)nb * 4 * 5 * 4);
  hipMemcpyToSymbol(HIP_SYMBOL(g_w4_stamps), &st, sizeof(st));
  for (int it = 0; it < 8; ++it) {
    int rc = cram_gemm(x, K, w, K, o, N, M, N, K, CRAM_GEMM_STORE, CRAM_DTYPE_BF16, nullptr);
    if (rc) { printf("cram_gemm rc %d\n", rc); return 1; }
  }
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  hipEventRecord(a);
  cram_gemm(x, K, w, K, o, N, M, N, K, CRAM_GEMM_STORE, CRAM_DTYPE_BF16, nullptr);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  std::vector<unsigned> h((size_t)nb * 20);
  hipMemcpy(h.data(), st, h.size() * 4, hipMemcpyDeviceToHost);
  double s[5] = {0, 0, 0, 0, 0};
  for (size_t i = 0; i < (size_t)nb * 4; ++i)
    for (int j = 0; j < 5; ++j) s[j] += h[i * 5 + j];
  const double tiles = s[4];
  printf("M %d N %d K %d: %.3f ms (%.0f TFLOP/s, stamped build); per FULL K-tile (%.0f wave-tiles): whole %.0f cycles, "
         "B1 %.0f, B2 %.0f, B3 %.0f (MFMA floor 2048)\n", M, N, K, ms, 2.0 * M * N * K / ms / 1e9, tiles,
         s[3] / tiles, s[0] / tiles, s[1] / tiles, s[2] / tiles);
  return 0;
}
