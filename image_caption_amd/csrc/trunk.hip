// ResNet-101 trunk helpers (GridFeatureEncoder.cnn, grid:51 = torchvision resnet101 children[:-2]).
// Activations are NHWC bf16 hi/lo planes ([B][H][W][C], lo plane at +lo); every convolution is an
// MFMA GEMM over rows = output pixels (gemm.hip: the 3x3 and 7x7 convolutions as implicit GEMMs
// that gather their A tiles straight from the activation, BatchNorm as the fp32 scale/shift
// epilogue, the residual added from planes before the ReLU).  Here: the stem's input layout (the
// NCHW fp32 image as a zero-bordered NHWC4 plane pair), the stride-2 subsample feeding a 1x1
// downsample, the 3x3/2 max-pool, and the weight/BatchNorm packing.
#include "common.h"
#include "kernels.h"

namespace {

// planes [B][H][W][C] -> [B][H/2][W/2][C] (every other pixel: the 1x1 stride-2 downsample input)
__global__ void subsample2_kernel(const bf16_t* __restrict__ x, long xlo, int B, int H, int W, int C, bf16_t* out,
                                  long lo, int nsplit) {
  const int C8 = C / 8, OH = (H + 1) / 2, OW = (W + 1) / 2;
  const long total = (long)B * OH * OW * C8;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c8 = (int)(i % C8);
    const long r = i / C8;
    const int ow = (int)(r % OW), oh = (int)((r / OW) % OH), b = (int)(r / ((long)OH * OW));
    const long src = (((long)b * H + 2 * oh) * W + 2 * ow) * C + c8 * 8;
    const long dst = r * C + c8 * 8;
    *(u32x4*)(out + dst) = *(const u32x4*)(x + src);
    if (nsplit == 2) *(u32x4*)(out + dst + lo) = *(const u32x4*)(x + src + xlo);
  }
}

// 3x3 / stride 2 / pad 1 max-pool on planes (the value is hi + lo; -inf padding like torch);
// 8 channels per thread, 16-byte loads of each plane.  F16: fp16 planes (the ICAP_PREC_F16 trunk)
template <bool F16>
__global__ void maxpool3s2_kernel(const bf16_t* __restrict__ x, long xlo, int B, int H, int W, int C, int OH, int OW,
                                  bf16_t* out, long lo, int nsplit) {
  const int C8 = C / 8;
  const long total = (long)B * OH * OW * C8;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c8 = (int)(i % C8);
    const long r = i / C8;
    const int ow = (int)(r % OW), oh = (int)((r / OW) % OH), b = (int)(r / ((long)OH * OW));
    float m[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) m[e] = -INFINITY;
    for (int dy = 0; dy < 3; ++dy) {
      const int y = oh * 2 - 1 + dy;
      if (y < 0 || y >= H) continue;
      for (int dx = 0; dx < 3; ++dx) {
        const int xx = ow * 2 - 1 + dx;
        if (xx < 0 || xx >= W) continue;
        const long src = (((long)b * H + y) * W + xx) * C + c8 * 8;
        const u32x4 hv = *(const u32x4*)(x + src);
        u32x4 lv = {0, 0, 0, 0};
        if (nsplit == 2) lv = *(const u32x4*)(x + src + xlo);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const uint32_t hw = hv[e >> 1], lw = lv[e >> 1];
          const bf16_t hb = (bf16_t)(e & 1 ? hw >> 16 : hw & 0xffffu), lb = (bf16_t)(e & 1 ? lw >> 16 : lw & 0xffffu);
          const float v = F16 ? h2f(hb) + (nsplit == 2 ? h2f(lb) : 0.f) : bf2f(hb) + bf2f(lb);
          m[e] = fmaxf(m[e], v);
        }
      }
    }
    u32x4 ho, lo4;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      bf16_t h0, l0, h1, l1;
      if (F16) {
        split_h(m[2 * e], h0, l0);
        split_h(m[2 * e + 1], h1, l1);
      } else {
        split_bf(m[2 * e], h0, l0);
        split_bf(m[2 * e + 1], h1, l1);
      }
      ho[e] = (uint32_t)h0 | ((uint32_t)h1 << 16);
      lo4[e] = (uint32_t)l0 | ((uint32_t)l1 << 16);
    }
    *(u32x4*)(out + r * C + c8 * 8) = ho;
    if (nsplit == 2) *(u32x4*)(out + r * C + c8 * 8 + lo) = lo4;
  }
}

int grid_for(long n) { return (int)std::min<long>((n + 255) / 256, 65536); }

}  // namespace

hipError_t launch_subsample2(const bf16_t* x, long xlo, int B, int H, int W, int C, bf16_t* out, long lo, int nsplit,
                             hipStream_t s) {
  if (C % 8) return hipErrorInvalidValue;
  const long n = (long)B * ((H + 1) / 2) * ((W + 1) / 2) * (C / 8);
  hipLaunchKernelGGL(subsample2_kernel, dim3(grid_for(n)), dim3(256), 0, s, x, xlo, B, H, W, C, out, lo, nsplit);
  return hipGetLastError();
}

hipError_t launch_maxpool3s2(const bf16_t* x, long xlo, int B, int H, int W, int C, int OH, int OW, bf16_t* out,
                             long lo, int nsplit, hipStream_t s, bool f16) {
  if (C % 8) return hipErrorInvalidValue;
  const dim3 grid(grid_for((long)B * OH * OW * (C / 8)));
  if (f16)
    hipLaunchKernelGGL(maxpool3s2_kernel<true>, grid, dim3(256), 0, s, x, xlo, B, H, W, C, OH, OW, out, lo, nsplit);
  else
    hipLaunchKernelGGL(maxpool3s2_kernel<false>, grid, dim3(256), 0, s, x, xlo, B, H, W, C, OH, OW, out, lo, nsplit);
  return hipGetLastError();
}

namespace {

// torch conv weight [Cout][Cin][kh][kw] fp32 -> [Cout][Kp] bf16 (F16: fp16), k = (kh*kwp + kw)*cp + c, 0 on padding
template <bool F16>
__global__ void pack_conv_kernel(const float* __restrict__ w, int cout, int cin, int k, int cp, int kwp, int Kp,
                                 bf16_t* out) {
  const long total = (long)cout * Kp;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int kk = (int)(i % Kp);
    const long o = i / Kp;
    const int c = kk % cp, tap = kk / cp, kh = tap / kwp, kw = tap % kwp;
    float v = 0.f;
    if (c < cin && kw < k && kh < k) v = w[((o * cin + c) * k + kh) * k + kw];
    out[i] = cvt16<F16>(v);
  }
}

// (B,3,IH,IW) fp32 -> [B][IH + 2 border][IW + 2 border][4] planes, zero border and channel 3 (F16: fp16 planes)
template <bool F16>
__global__ void image_nhwc4_kernel(const float* __restrict__ img, int B, int IH, int IW, int border, bf16_t* out,
                                   long lo, int nsplit) {
  const int HP = IH + 2 * border, WP = IW + 2 * border;
  const long total = (long)B * HP * WP;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int x = (int)(i % WP) - border, y = (int)((i / WP) % HP) - border;
    const long b = i / ((long)HP * WP);
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    if (y >= 0 && y < IH && x >= 0 && x < IW)
#pragma unroll
      for (int c = 0; c < 3; ++c) v[c] = img[((b * 3 + c) * IH + y) * IW + x];
    bf16_t h[4], l[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      if (F16) split_h(v[c], h[c], l[c]);
      else split_bf(v[c], h[c], l[c]);
    }
    u32x2 hv = {(uint32_t)h[0] | ((uint32_t)h[1] << 16), (uint32_t)h[2] | ((uint32_t)h[3] << 16)};
    *(u32x2*)(out + i * 4) = hv;
    if (nsplit == 2) {
      u32x2 lv = {(uint32_t)l[0] | ((uint32_t)l[1] << 16), (uint32_t)l[2] | ((uint32_t)l[3] << 16)};
      *(u32x2*)(out + i * 4 + lo) = lv;
    }
  }
}

// eval BatchNorm as y = x * scale + shift: scale = gamma / sqrt(var + eps), shift = beta - mean * scale
__global__ void bn_fold_kernel(const float* g, const float* b, const float* mean, const float* var, int C, float eps,
                               float* scale, float* shift) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float sc = g[c] / sqrtf(var[c] + eps);
  scale[c] = sc;
  shift[c] = b[c] - mean[c] * sc;
}


// ---- train-mode BatchNorm (GridFeatureEncoder.cnn under module.train(): the reference's SCST step,
// scst_loss:161 / :213).  The convolution's GEMM writes its raw output y as planes; bn_stats sums y and y^2
// per channel over all M = B*H*W rows (double accumulators, fixed reduction order: deterministic),
// bn_finalize turns them into the batch mean / biased variance, the fp32 scale / shift of
// y * scale + shift = (y - mean) / sqrt(var + eps) * gamma + beta, and updates the running statistics as
// torch's BatchNorm2d does (momentum, unbiased variance M / (M - 1)); bn_apply normalises in place, adds
// the residual planes and applies the ReLU (the eval epilogue's order).

// block = 16 column groups of 4 channels (64 channels) x 16 row lanes; part[chunk][C][2] doubles
__global__ __launch_bounds__(256) void bn_stats_kernel(const bf16_t* __restrict__ y, long lo, long M, int C,
                                                       long rows_per_chunk, double* part) {
  __shared__ double red[16][64][2];
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  const int c0 = blockIdx.x * 64 + tx * 4;
  const long r0 = blockIdx.y * rows_per_chunk, r1 = min(M, r0 + rows_per_chunk);
  double s[4] = {0, 0, 0, 0}, q[4] = {0, 0, 0, 0};
  for (long r = r0 + ty; r < r1; r += 16) {
    const u32x2 h = *(const u32x2*)(y + r * C + c0), l = *(const u32x2*)(y + r * C + c0 + lo);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t wh = h[k >> 1] >> ((k & 1) * 16), wl = l[k >> 1] >> ((k & 1) * 16);
      const double v = (double)(bf2f((bf16_t)(wh & 0xffff)) + bf2f((bf16_t)(wl & 0xffff)));
      s[k] += v;
      q[k] += v * v;
    }
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    red[ty][tx * 4 + k][0] = s[k];
    red[ty][tx * 4 + k][1] = q[k];
  }
  __syncthreads();
  if (threadIdx.x < 128) {  // channel threadIdx.x / 2, sum (0) or squares (1), rows lanes in order
    const int ch = threadIdx.x >> 1, w = threadIdx.x & 1;
    double t = 0;
    for (int i = 0; i < 16; ++i) t += red[i][ch][w];
    part[((long)blockIdx.y * C + blockIdx.x * 64 + ch) * 2 + w] = t;
  }
}

__global__ void bn_finalize_kernel(const double* __restrict__ part, int nchunks, int C, long M, const float* gamma,
                                   const float* beta, float* run_mean, float* run_var, float momentum, float eps,
                                   float* scale, float* shift) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double s = 0, q = 0;
  for (int i = 0; i < nchunks; ++i) {
    s += part[((long)i * C + c) * 2];
    q += part[((long)i * C + c) * 2 + 1];
  }
  const double mean = s / (double)M, var = fmax(q / (double)M - mean * mean, 0.0);
  const float invstd = 1.0f / sqrtf((float)var + eps);
  const float sc = gamma[c] * invstd;
  scale[c] = sc;
  shift[c] = beta[c] - (float)mean * sc;
  run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * (float)mean;
  run_var[c] = (1.f - momentum) * run_var[c] + momentum * (float)(var * (double)M / (double)(M - 1));
}

// in place: y = relu?(y * scale + shift (+ res)), 4 channels per thread
__global__ void bn_apply_kernel(bf16_t* y, long lo, long M, int C, const float* __restrict__ scale,
                                const float* __restrict__ shift, const bf16_t* __restrict__ res, long res_lo,
                                int relu) {
  const long total = M * C / 4;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c0 = (int)((i * 4) % C);
    const u32x2 h = *(const u32x2*)(y + i * 4), l = *(const u32x2*)(y + i * 4 + lo);
    u32x2 rh = {0, 0}, rl = {0, 0};
    if (res) {
      rh = *(const u32x2*)(res + i * 4);
      rl = *(const u32x2*)(res + i * 4 + res_lo);
    }
    const f32x4 sc = *(const f32x4*)(scale + c0), sh = *(const f32x4*)(shift + c0);
    bf16_t oh[4], ol[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int sft = (k & 1) * 16;
      float v = (bf2f((bf16_t)((h[k >> 1] >> sft) & 0xffff)) + bf2f((bf16_t)((l[k >> 1] >> sft) & 0xffff))) * sc[k] +
                sh[k];
      if (res) v += bf2f((bf16_t)((rh[k >> 1] >> sft) & 0xffff)) + bf2f((bf16_t)((rl[k >> 1] >> sft) & 0xffff));
      if (relu) v = fmaxf(v, 0.f);
      split_bf(v, oh[k], ol[k]);
    }
    *(u32x2*)(y + i * 4) = (u32x2){(uint32_t)oh[0] | ((uint32_t)oh[1] << 16), (uint32_t)oh[2] | ((uint32_t)oh[3] << 16)};
    *(u32x2*)(y + i * 4 + lo) =
        (u32x2){(uint32_t)ol[0] | ((uint32_t)ol[1] << 16), (uint32_t)ol[2] | ((uint32_t)ol[3] << 16)};
  }
}

}  // namespace

hipError_t launch_pack_conv(const float* w, int cout, int cin, int k, int cp, int kwp, int Kp, bf16_t* out,
                            hipStream_t s, bool f16) {
  if (cp < cin || kwp < k || Kp < k * kwp * cp) return hipErrorInvalidValue;
  const dim3 grid(grid_for((long)cout * Kp));
  if (f16) hipLaunchKernelGGL(pack_conv_kernel<true>, grid, dim3(256), 0, s, w, cout, cin, k, cp, kwp, Kp, out);
  else hipLaunchKernelGGL(pack_conv_kernel<false>, grid, dim3(256), 0, s, w, cout, cin, k, cp, kwp, Kp, out);
  return hipGetLastError();
}

hipError_t launch_image_nhwc4(const float* img, int B, int IH, int IW, int border, bf16_t* out, long lo, int nsplit,
                              hipStream_t s, bool f16) {
  const long HP = IH + 2 * border, WP = IW + 2 * border;
  const dim3 grid(grid_for(B * HP * WP));
  if (f16)
    hipLaunchKernelGGL(image_nhwc4_kernel<true>, grid, dim3(256), 0, s, img, B, IH, IW, border, out, lo, nsplit);
  else
    hipLaunchKernelGGL(image_nhwc4_kernel<false>, grid, dim3(256), 0, s, img, B, IH, IW, border, out, lo, nsplit);
  return hipGetLastError();
}

hipError_t launch_bn_fold(const float* g, const float* b, const float* mean, const float* var, int C, float eps,
                          float* scale, float* shift, hipStream_t s) {
  hipLaunchKernelGGL(bn_fold_kernel, dim3((C + 255) / 256), dim3(256), 0, s, g, b, mean, var, C, eps, scale, shift);
  return hipGetLastError();
}

int bn_stats_chunks(long M, int C) {
  // ~1024 blocks over the (64-channel group, row chunk) grid, >= 256 rows per chunk
  const long groups = C / 64;
  long n = std::max(1L, 1024 / groups);
  n = std::min(n, std::max(1L, M / 256));
  return (int)n;
}

hipError_t launch_bn_train(bf16_t* y, long lo, long M, int C, const float* gamma, const float* beta, float* run_mean,
                           float* run_var, float momentum, float eps, const bf16_t* res, long res_lo, int relu,
                           double* part, float* scale, float* shift, hipStream_t s) {
  if (M < 2 || C % 64) return hipErrorInvalidValue;
  const int nch = bn_stats_chunks(M, C);
  const long rpc = (M + nch - 1) / nch;
  hipLaunchKernelGGL(bn_stats_kernel, dim3(C / 64, nch), dim3(256), 0, s, y, lo, M, C, rpc, part);
  hipLaunchKernelGGL(bn_finalize_kernel, dim3((C + 255) / 256), dim3(256), 0, s, part, nch, C, M, gamma, beta,
                     run_mean, run_var, momentum, eps, scale, shift);
  hipLaunchKernelGGL(bn_apply_kernel, dim3(grid_for(M * C / 4)), dim3(256), 0, s, y, lo, M, C, scale, shift, res,
                     res_lo, relu);
  return hipGetLastError();
}
