// hipBLASLt on the ViT residual GEMMs (tools probe, round 5): D = A W^T + b + C with fp16 A / W, fp32 C = D (the
// residual stream, beta = 1, bias epilogue) at M = 50432 (B = 256 x 197 tokens).  Prints the heuristic's first
// algorithms' times for out-proj (K = 768) and MLP-2 (K = 3072), N = 768.
// build: hipcc --offload-arch=gfx950 -O2 tools/probe_blaslt.cpp -lhipblaslt -o tools/probe_blaslt
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    auto e_ = (x);                                                             \
    if ((int)e_ != 0) {                                                        \
      printf("error %d at %s:%d (%s)\n", (int)e_, __FILE__, __LINE__, #x);    \
      return 1;                                                                \
    }                                                                          \
  } while (0)

static int run(hipblasLtHandle_t lt, int M, int N, int K, int outf16, void* ws, size_t wsz) {
  void *A, *W, *C, *bias;
  CK(hipMalloc(&A, (size_t)M * K * 2));
  CK(hipMalloc(&W, (size_t)N * K * 2));
  CK(hipMalloc(&C, (size_t)M * N * 4));
  CK(hipMalloc(&bias, (size_t)N * 4));
  {  // random operands (constant ones run at a higher clock): A uniform(-0.5, 0.5), W ~ uniform / sqrt(K)
    std::vector<_Float16> h((size_t)M * K);
    uint32_t x = 12345;
    auto rnd = [&] { x = x * 1664525u + 1013904223u; return (float)(x >> 8) / 16777216.f - 0.5f; };
    for (auto& v : h) v = (_Float16)rnd();
    CK(hipMemcpy(A, h.data(), h.size() * 2, hipMemcpyHostToDevice));
    h.resize((size_t)N * K);
    for (auto& v : h) v = (_Float16)(rnd() * 3.4f / sqrtf((float)K));
    CK(hipMemcpy(W, h.data(), h.size() * 2, hipMemcpyHostToDevice));
  }
  CK(hipMemset(C, 0, (size_t)M * N * 4));
  CK(hipMemset(bias, 0, (size_t)N * 4));
  const hipDataType ct = outf16 ? HIP_R_16F : HIP_R_32F;
  hipblasLtMatmulDesc_t desc;
  CK(hipblasLtMatmulDescCreate(&desc, HIPBLAS_COMPUTE_32F, HIP_R_32F));
  hipblasOperation_t ta = HIPBLAS_OP_T, tb = HIPBLAS_OP_N;
  CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta)));
  CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb)));
  hipblasLtEpilogue_t epi = HIPBLASLT_EPILOGUE_BIAS;
  CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &epi, sizeof(epi)));
  CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias, sizeof(bias)));
  hipDataType bt = HIP_R_32F;
  CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt)));
  hipblasLtMatrixLayout_t la, lb, lc;
  CK(hipblasLtMatrixLayoutCreate(&la, HIP_R_16F, K, N, K));  // W stored K x N (col-major), op T
  CK(hipblasLtMatrixLayoutCreate(&lb, HIP_R_16F, K, M, K));  // A stored K x M (col-major)
  CK(hipblasLtMatrixLayoutCreate(&lc, ct, N, M, N));          // C = D: N x M (col-major) = row-major [M][N]
  hipblasLtMatmulPreference_t pref;
  CK(hipblasLtMatmulPreferenceCreate(&pref));
  CK(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsz, sizeof(wsz)));
  hipblasLtMatmulHeuristicResult_t res[8];
  int nres = 0;
  CK(hipblasLtMatmulAlgoGetHeuristic(lt, desc, la, lb, lc, lc, pref, 8, res, &nres));
  const float alpha = 1.f, beta = outf16 ? 0.f : 1.f;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int a = 0; a < nres; ++a) {
    for (int i = 0; i < 3; ++i)
      CK(hipblasLtMatmul(lt, desc, &alpha, W, la, A, lb, &beta, C, lc, C, lc, &res[a].algo, ws, wsz, 0));
    const int it = 20;
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < it; ++i)
      CK(hipblasLtMatmul(lt, desc, &alpha, W, la, A, lb, &beta, C, lc, C, lc, &res[a].algo, ws, wsz, 0));
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1000.0 / it;
    printf("M %d N %d K %d out %s beta %.0f algo %d: %.1f us  %.1f TFLOP/s\n", M, N, K, outf16 ? "f16" : "f32", beta, a,
           us, 2.0 * M * N * K / us / 1e6);
  }
  hipFree(A);
  hipFree(W);
  hipFree(C);
  hipFree(bias);
  return 0;
}

int main() {
  hipblasLtHandle_t lt;
  CK(hipblasLtCreate(&lt));
  const size_t wsz = 64 << 20;
  void* ws;
  CK(hipMalloc(&ws, wsz));
  const int M = 50432;
  for (int K : {768, 3072}) {
    if (run(lt, M, 768, K, 0, ws, wsz)) return 1;
    if (run(lt, M, 768, K, 1, ws, wsz)) return 1;
  }
  return 0;
}
