// Per-kernel cost floor under hipGraph replay: 100 back-to-back launches captured in one graph,
// replayed, wall time / 100.  Kernels: empty; one 16-B load + store per thread; an LN-shaped row
// kernel (256 rows x 512 fp32, 4 partial slabs + x in, x + bf16 plane out).
// Build: hipcc --offload-arch=gfx950 -O3 tools/probe_small.hip -o tools/probe_small
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1); } } while (0)
typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void k_empty(float* p) {
  if (p == nullptr) p[threadIdx.x] = 0;
}
__global__ void k_copy(const f32x4* __restrict__ a, f32x4* __restrict__ b, long n) {
  const long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (i < n) b[i] = a[i] * 1.5f;
}
__global__ __launch_bounds__(128) void k_ln(float* __restrict__ x, const float* __restrict__ parts, int nparts) {
  __shared__ float red[2];
  const int row = blockIdx.x, col = threadIdx.x * 4;
  f32x4 v = *(const f32x4*)(x + row * 512 + col);
  f32x4 pp[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) pp[s] = *(const f32x4*)(parts + s * 131072 + row * 512 + col);
#pragma unroll
  for (int s = 0; s < 4; ++s) v += pp[s];
  float sm = v[0] + v[1] + v[2] + v[3];
  for (int o = 32; o; o >>= 1) sm += __shfl_xor(sm, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = sm;
  __syncthreads();
  const float mean = (red[0] + red[1]) / 512.f;
  *(f32x4*)(x + row * 512 + col) = (v - mean) * 0.999f;
}

// one function for both bodies: is the alternation cost tied to switching kernel objects?
__global__ __launch_bounds__(256) void k_multi(int mode, float* __restrict__ x, const float* __restrict__ parts,
                                               const f32x4* __restrict__ a, f32x4* __restrict__ b, long n) {
  if (mode == 0) {
    const long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (i < n) b[i] = a[i] * 1.5f;
    return;
  }
  __shared__ float red[2];
  const int row = blockIdx.x, col = threadIdx.x * 4;
  f32x4 v = *(const f32x4*)(x + row * 512 + col);
  f32x4 pp[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) pp[s] = *(const f32x4*)(parts + s * 131072 + row * 512 + col);
#pragma unroll
  for (int s = 0; s < 4; ++s) v += pp[s];
  float sm = v[0] + v[1] + v[2] + v[3];
  for (int o = 32; o; o >>= 1) sm += __shfl_xor(sm, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = sm;
  __syncthreads();
  const float mean = (red[0] + red[1]) / 512.f;
  *(f32x4*)(x + row * 512 + col) = (v - mean) * 0.999f;
}

template <class F>
float graph_time(F launch, hipStream_t s, int n = 100) {
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
  for (int i = 0; i < n; ++i) launch();
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  CK(hipGraphLaunch(ge, s));
  CK(hipStreamSynchronize(s));
  CK(hipEventRecord(a, s));
  for (int r = 0; r < 5; ++r) CK(hipGraphLaunch(ge, s));
  CK(hipEventRecord(b, s));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms * 1e3f / (5 * n);
}

int main() {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  float *x, *parts, *buf;
  CK(hipMalloc(&x, 256 * 512 * 4));
  CK(hipMalloc(&parts, 8 * 131072 * 4));
  CK(hipMalloc(&buf, 64 << 20));
  CK(hipMemset(x, 0, 256 * 512 * 4));
  CK(hipMemset(parts, 0, 8 * 131072 * 4));
  CK(hipMemset(buf, 0, 64 << 20));
  for (int blocks : {1, 64, 256, 1024, 4096}) {
    const float t = graph_time([&] { hipLaunchKernelGGL(k_empty, dim3(blocks), dim3(256), 0, s, (float*)nullptr + 1); }, s);
    printf("empty       blocks %5d : %6.2f us/kernel\n", blocks, t);
  }
  for (long bytes : {64L << 10, 1L << 20, 4L << 20, 16L << 20}) {
    const long n = bytes / 16;
    const float t = graph_time([&] {
      hipLaunchKernelGGL(k_copy, dim3((n + 255) / 256), dim3(256), 0, s, (const f32x4*)buf, (f32x4*)(buf + (32 << 18)), n);
    }, s);
    printf("copy %6ld KiB : %6.2f us/kernel\n", bytes >> 10, t);
  }
  {
    const float t = graph_time([&] { hipLaunchKernelGGL(k_ln, dim3(256), dim3(128), 0, s, x, parts, 4); }, s);
    printf("ln 256 rows : %6.2f us/kernel\n", t);
  }
  // ping-pong chains: kernel i reads what kernel i-1 wrote (dependent) or a fixed buffer (independent)
  for (long bytes : {256L << 10, 1L << 20, 2L << 20, 8L << 20}) {
    const long n = bytes / 16;
    f32x4* A = (f32x4*)buf;
    f32x4* B = (f32x4*)(buf + (16 << 18));
    f32x4* C = (f32x4*)(buf + (32 << 18));
    int i = 0;
    const float dep = graph_time([&] {
      f32x4* src = (i & 1) ? B : A;
      f32x4* dst = (i & 1) ? A : B;
      ++i;
      hipLaunchKernelGGL(k_copy, dim3((n + 255) / 256), dim3(256), 0, s, (const f32x4*)src, dst, n);
    }, s);
    i = 0;
    const float ind = graph_time([&] {
      f32x4* dst = (i & 1) ? A : B;
      ++i;
      hipLaunchKernelGGL(k_copy, dim3((n + 255) / 256), dim3(256), 0, s, (const f32x4*)C, dst, n);
    }, s);
    printf("chain %5ld KiB : dependent %6.2f  independent %6.2f us/kernel\n", bytes >> 10, dep, ind);
  }
  {  // LN fed by a producer that writes its partial slabs (2 MiB) from a fixed source
    const float t = graph_time([&] {
      hipLaunchKernelGGL(k_copy, dim3(512), dim3(256), 0, s, (const f32x4*)buf, (f32x4*)parts, 131072L);
      hipLaunchKernelGGL(k_ln, dim3(256), dim3(128), 0, s, x, parts, 4);
    }, s, 50);
    printf("producer+ln pair : %6.2f us/kernel\n", t);
  }
  {
    const long n = 65536;  // 1 MiB
    f32x4* A = (f32x4*)buf;
    f32x4* B = (f32x4*)(buf + (16 << 18));
    float t = graph_time([&] {
      hipLaunchKernelGGL(k_copy, dim3(n / 256), dim3(256), 0, s, (const f32x4*)A, B, n);
      hipLaunchKernelGGL(k_copy, dim3(n / 128), dim3(128), 0, s, (const f32x4*)A, B + n, n);
    }, s, 50);
    printf("alt copy256/copy128 : %6.2f us/kernel\n", t);
    t = graph_time([&] {
      hipLaunchKernelGGL(k_copy, dim3(n / 256), dim3(256), 0, s, (const f32x4*)A, B, n);
      hipLaunchKernelGGL(k_empty, dim3(256), dim3(256), 0, s, (float*)nullptr + 1);
    }, s, 50);
    printf("alt copy/empty : %6.2f us/kernel\n", t);
    t = graph_time([&] {
      hipLaunchKernelGGL(k_ln, dim3(256), dim3(128), 0, s, x, parts, 4);
      hipLaunchKernelGGL(k_empty, dim3(256), dim3(256), 0, s, (float*)nullptr + 1);
    }, s, 50);
    printf("alt ln/empty : %6.2f us/kernel\n", t);
    t = graph_time([&] {
      hipLaunchKernelGGL(k_ln, dim3(256), dim3(128), 0, s, x, parts, 4);
      hipLaunchKernelGGL(k_copy, dim3(n / 256), dim3(256), 0, s, (const f32x4*)A, B, n);
    }, s, 50);
    printf("alt ln/copy(indep) : %6.2f us/kernel\n", t);
    t = graph_time([&] {
      hipLaunchKernelGGL(k_multi, dim3(256), dim3(128), 0, s, 1, x, parts, (const f32x4*)A, B, n);
      hipLaunchKernelGGL(k_multi, dim3(n / 256), dim3(256), 0, s, 0, x, parts, (const f32x4*)A, B, n);
    }, s, 50);
    printf("alt ln/copy merged kernel : %6.2f us/kernel\n", t);
    t = graph_time([&] {
      hipLaunchKernelGGL(k_multi, dim3(256), dim3(128), 0, s, 1, x, parts, (const f32x4*)A, B, n);
    }, s, 100);
    printf("merged kernel ln only : %6.2f us/kernel\n", t);
    t = graph_time([&] {
      hipLaunchKernelGGL(k_multi, dim3(n / 256), dim3(256), 0, s, 0, x, parts, (const f32x4*)A, B, n);
    }, s, 100);
    printf("merged kernel copy only : %6.2f us/kernel\n", t);
    t = graph_time([&] {
      hipLaunchKernelGGL(k_copy, dim3(n / 256), dim3(256), 0, s, (const f32x4*)A, B, n);
    }, s, 100);
    printf("copy 1MiB only : %6.2f us/kernel\n", t);
    // what changes between consecutive dispatches makes them slow: grid size, LDS size, mode arg
    t = graph_time([&] {
      hipLaunchKernelGGL(k_copy, dim3(n / 256), dim3(256), 0, s, (const f32x4*)A, B, n);
      hipLaunchKernelGGL(k_copy, dim3(n / 512), dim3(256), 0, s, (const f32x4*)A, B, n / 2);
    }, s, 50);
    printf("alt copy grid 256 / 128 blocks (same block size) : %6.2f us/kernel\n", t);
    t = graph_time([&] {
      hipLaunchKernelGGL(k_copy, dim3(n / 256), dim3(256), 0, s, (const f32x4*)A, B, n);
      hipLaunchKernelGGL(k_copy, dim3(n / 256), dim3(256), 8192, s, (const f32x4*)A, B, n);
    }, s, 50);
    printf("alt copy dyn LDS 0 / 8 KiB : %6.2f us/kernel\n", t);
    t = graph_time([&] {
      hipLaunchKernelGGL(k_multi, dim3(256), dim3(256), 0, s, 1, x, parts, (const f32x4*)A, B, n);
      hipLaunchKernelGGL(k_multi, dim3(n / 256), dim3(256), 0, s, 0, x, parts, (const f32x4*)A, B, n);
    }, s, 50);
    printf("alt merged ln/copy, both 256 threads : %6.2f us/kernel\n", t);
    t = graph_time([&] {
      hipLaunchKernelGGL(k_multi, dim3(256), dim3(256), 0, s, 1, x, parts, (const f32x4*)A, B, n);
      hipLaunchKernelGGL(k_multi, dim3(256), dim3(256), 0, s, 0, x, parts, (const f32x4*)A, B, 256 * 256);
    }, s, 50);
    printf("alt merged ln/copy, same grid and block : %6.2f us/kernel\n", t);
    t = graph_time([&] {
      hipLaunchKernelGGL(k_copy, dim3(256), dim3(256), 0, s, (const f32x4*)A, B, 256 * 256);
      hipLaunchKernelGGL(k_empty, dim3(256), dim3(256), 0, s, (float*)nullptr + 1);
    }, s, 50);
    printf("alt copy/empty, same grid and block : %6.2f us/kernel\n", t);
    // stream launches (no graph) for the ln/copy alternation
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipEventRecord(a, s));
    for (int r = 0; r < 250; ++r) {
      hipLaunchKernelGGL(k_ln, dim3(256), dim3(128), 0, s, x, parts, 4);
      hipLaunchKernelGGL(k_copy, dim3(n / 256), dim3(256), 0, s, (const f32x4*)A, B, n);
    }
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    printf("alt ln/copy stream : %6.2f us/kernel\n", ms * 1e3f / 500);
  }
  return 0;
}
