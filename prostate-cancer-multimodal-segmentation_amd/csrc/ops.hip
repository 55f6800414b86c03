// Bandwidth-bound kernels of the U-Net step (NDHWC, gfx950): input layout pack,
// BatchNorm3d (train/eval) + ReLU forward/backward, MaxPool3d(2) forward/backward,
// the 1x1x1 output conv, DiceLoss / BCEDiceLoss forward/backward, flat Adam.
//
// Reference ops replaced (paths relative to the reference repo):
//   BatchNorm3d + ReLU(inplace)   models/unet3d.py:31-39
//   MaxPool3d(2)                  models/unet3d.py:80
//   outc Conv3d(64, ncls, 1)      models/unet3d.py:222
//   DiceLoss / BCEDiceLoss        utils/losses.py:44-92, 124-152
//   optim.Adam(wd=1e-5, coupled)  utils/trainer.py:113-117
// Every per-channel statistic is a two-level reduction: fp32 per-block partials written
// to a [rows][C][2] buffer, combined in fp64 in a fixed order (run-to-run reproducible).
#include "common.h"
#include "pcms_hip.h"
#include <algorithm>

namespace {

constexpr int TPB = 256;

inline int grid_for(long work, int per_block, int cap = 8192) {
  return (int)std::max<long>(1, std::min<long>(cap, (work + per_block - 1) / per_block));
}

// ---------------- input: NCDHW fp32 (N, Cin, V) -> NDHWC T (N, V, Cp) ----------------
template <typename T>
__global__ void pack_input_kernel(const float* in, T* out, int N, int Cin, long V, int Cp) {
  const long total = (long)N * V;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long n = i / V, v = i % V;
    for (int c = 0; c < Cp; ++c) {
      const float x = c < Cin ? in[(n * Cin + c) * V + v] : 0.f;
      Elem<T>::st(out + i * Cp + c, x);
    }
  }
}

// the same with 4 voxels per thread (V % 4 == 0, Cin <= Cp == 8): one 16-B load per input
// channel, one 16-B (bf16) / two 16-B (fp32) stores per voxel
template <typename T>
__global__ void __launch_bounds__(256) pack_input4_kernel(const float* in, T* out, int N, int Cin, long V) {
  const long quads = (long)N * V / 4;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < quads; i += (long)gridDim.x * blockDim.x) {
    const long n = (4 * i) / V, v = (4 * i) % V;
    f32x4_t x[8];
#pragma unroll
    for (int c = 0; c < 8; ++c)
      x[c] = c < Cin ? __builtin_nontemporal_load(reinterpret_cast<const f32x4_t*>(in + (n * Cin + c) * V + v))
                     : (f32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if constexpr (sizeof(T) == 2) {
        const u32x4_t o = {pack_bf16x2(x[0][k], x[1][k]), pack_bf16x2(x[2][k], x[3][k]),
                           pack_bf16x2(x[4][k], x[5][k]), pack_bf16x2(x[6][k], x[7][k])};
        *reinterpret_cast<u32x4_t*>(out + (4 * i + k) * 8) = o;
      } else {
        *reinterpret_cast<f32x4_t*>(out + (4 * i + k) * 8) = (f32x4_t){x[0][k], x[1][k], x[2][k], x[3][k]};
        *reinterpret_cast<f32x4_t*>(out + (4 * i + k) * 8 + 4) = (f32x4_t){x[4][k], x[5][k], x[6][k], x[7][k]};
      }
    }
  }
}

// ---------------- BatchNorm statistics ----------------
// Stage 1: fp32 partial rows [rows][C][2] -> fp64 column sums [RB][C][2] (RB row groups).
// block = 256 threads = 4 row lanes x 64 channels; grid = (ceil(C / 64), RB).
// cnt != NULL: rows are (sum, M2 about the row mean) with per-row voxel counts cnt[rows];
// column 2 then accumulates M2 + sum^2 / count (= the row's sum of squares, formed in fp64).
constexpr int kRB = 64;
__global__ void __launch_bounds__(256) colsum2_kernel(const float* part, int rows, int C, const float* cnt,
                                                      double* out) {
  __shared__ double red[4][64][2];
  const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  double s1 = 0.0, s2 = 0.0;
  auto add = [&](const float2 v, int r) {
    s1 += (double)v.x;
    if (cnt) {
      const double n = (double)cnt[r];
      s2 += (double)v.y + (n > 0.0 ? (double)v.x * (double)v.x / n : 0.0);
    } else {
      s2 += (double)v.y;
    }
  };
  if (c < C) {
    // rows r, r + 256, ... added in that order, four rows' loads in flight per trip
    constexpr int RS = kRB * 4;
    int r = blockIdx.y * 4 + rl;
    for (; r + 3 * RS < rows; r += 4 * RS) {
      float2 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const float2*>(part + ((long)(r + u * RS) * C + c) * 2);
#pragma unroll
      for (int u = 0; u < 4; ++u) add(v[u], r + u * RS);
    }
    for (; r < rows; r += RS) add(*reinterpret_cast<const float2*>(part + ((long)r * C + c) * 2), r);
  }
  red[rl][cl][0] = s1;
  red[rl][cl][1] = s2;
  __syncthreads();
  if (rl == 0 && c < C) {
    for (int g = 1; g < 4; ++g) { s1 += red[g][cl][0]; s2 += red[g][cl][1]; }
    out[((long)blockIdx.y * C + c) * 2] = s1;
    out[((long)blockIdx.y * C + c) * 2 + 1] = s2;
  }
}

// the kRB row sums of channel c, added in row order; 16 rows' loads in flight at a time (one
// thread per channel: a dependent load -> add chain made each finalize launch ~8 us)
__device__ __forceinline__ void colsum_final(const double* ws, int C, int c, double& s1, double& s2) {
  s1 = 0.0; s2 = 0.0;
  const double2* p = reinterpret_cast<const double2*>(ws) + c;
#pragma unroll
  for (int r0 = 0; r0 < kRB; r0 += 16) {
    double2 v[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = p[(long)(r0 + i) * C];
#pragma unroll
    for (int i = 0; i < 16; ++i) { s1 += v[i].x; s2 += v[i].y; }
  }
}

// Stage 2: -> mean/invstd/scale/shift (+ running stats when training)
__device__ __forceinline__ void bn_finalize_one(int c, double s1, double s2, double count, const float* gamma,
                                                const float* beta, float* rmean, float* rvar, float momentum,
                                                float eps, float* scale, float* shift, float* mean_out,
                                                float* invstd_out) {
  const double mean = s1 / count;
  double var = s2 / count - mean * mean;
  if (var < 0) var = 0;
  const double inv = 1.0 / sqrt(var + (double)eps);
  scale[c] = (float)((double)gamma[c] * inv);
  shift[c] = (float)((double)beta[c] - mean * (double)gamma[c] * inv);
  mean_out[c] = (float)mean;
  invstd_out[c] = (float)inv;
  if (rmean) {
    const double unb = count > 1 ? var * count / (count - 1) : var;
    rmean[c] = (float)((1.0 - momentum) * (double)rmean[c] + momentum * mean);
    rvar[c] = (float)((1.0 - momentum) * (double)rvar[c] + momentum * unb);
  }
}
__global__ void bn_finalize_kernel(const double* ws, int C, double count, const float* gamma, const float* beta,
                                   float* rmean, float* rvar, long long* nbt, float momentum, float eps,
                                   float* scale, float* shift, float* mean_out, float* invstd_out) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (nbt && c == 0) *nbt += 1;
  if (c >= C) return;
  double s1, s2;
  colsum_final(ws, C, c, s1, s2);
  bn_finalize_one(c, s1, s2, count, gamma, beta, rmean, rvar, momentum, eps, scale, shift, mean_out, invstd_out);
}

// Eval-mode BatchNorm folded into the conv before it (UNet3D.predict / inference,
// models/unet3d.py:298-344: BN over the running statistics is an affine map per output
// channel): w' = w sc, b' = b sc + sh, sc / sh in fp64 as bn_eval_coeffs_kernel forms them.
// w: [Cout][K] fp32 (torch layout, K = Cin x 27).
__global__ void bn_fold_kernel(const float* w, const float* b, const float* gamma, const float* beta,
                               const float* rmean, const float* rvar, float eps, int Cout, long K, float* wo,
                               float* bo) {
  const int co = blockIdx.y;
  const double inv = 1.0 / sqrt((double)rvar[co] + (double)eps);
  const double sc = (double)gamma[co] * inv;
  const float scf = (float)sc;
  for (long k = blockIdx.x * (long)blockDim.x + threadIdx.x; k < K; k += (long)gridDim.x * blockDim.x)
    wo[(long)co * K + k] = w[(long)co * K + k] * scf;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    const double sh = (double)beta[co] - (double)rmean[co] * sc;
    bo[co] = (float)((b ? (double)b[co] : 0.0) * sc + sh);
  }
}

__global__ void bn_eval_coeffs_kernel(const float* gamma, const float* beta, const float* rmean,
                                      const float* rvar, float eps, int C, float* scale, float* shift) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const double inv = 1.0 / sqrt((double)rvar[c] + (double)eps);
  scale[c] = (float)((double)gamma[c] * inv);
  shift[c] = (float)((double)beta[c] - (double)rmean[c] * (double)gamma[c] * inv);
}

// a = relu(y * scale[c] + shift[c]); 16-byte vectors.  Block = (256 / CG) voxel lanes x
// CG channel groups, so every thread keeps its VEC channels' coefficients in registers.
// NT: non-temporal loads and stores for tensors far larger than the Infinity Cache
// (measured: level-0 bn_relu 90 -> 87 us; walking the voxels in reverse to catch the
// producer's cached tail bought nothing)
template <typename T, bool NT>
__global__ void __launch_bounds__(TPB) bn_relu_kernel(const T* y, T* a, const float* scale, const float* shift,
                                                      int C, long nvox) {
  constexpr int VEC = Elem<T>::kVec;
  const int CG = C / VEC;
  const int cg = threadIdx.x % CG, vl = threadIdx.x / CG, VL = TPB / CG;
  const int c0 = cg * VEC;
  float sc[VEC], sh[VEC];
#pragma unroll
  for (int j = 0; j < VEC; ++j) { sc[j] = scale[c0 + j]; sh[j] = shift[c0 + j]; }
  for (long v = (long)blockIdx.x * VL + vl; v < nvox; v += (long)gridDim.x * VL) {
    float x[VEC];
    ld16<NT>(y + v * C + c0, x);
#pragma unroll
    for (int j = 0; j < VEC; ++j) x[j] = bn_relu1(x[j], sc[j], sh[j]);
    st16<NT>(a + v * C + c0, x);
  }
}

// BN+ReLU backward, pass 1: per-block partial sums of g and g*xhat, g = da * [a > 0].
// Block: 256 threads = (256 / C8) voxel lanes x C8 channel groups of VEC channels.
template <typename T, bool NT>
__global__ void __launch_bounds__(TPB) bn_relu_bwd_reduce_kernel(
    const T* da, const T* y, const float* scale, const float* shift, const float* mean,
    const float* invstd, float* part, int C, long nvox) {
  constexpr int VEC = Elem<T>::kVec;
  __shared__ float red[TPB * VEC * 2];
  const int CG = C / VEC;
  const int cg = threadIdx.x % CG, vl = threadIdx.x / CG, VL = TPB / CG;
  const int c0 = cg * VEC;
  float sc[VEC], sh[VEC], mu[VEC], is[VEC], sg[VEC], sgx[VEC];
#pragma unroll
  for (int j = 0; j < VEC; ++j) {
    sc[j] = scale[c0 + j]; sh[j] = shift[c0 + j]; mu[j] = mean[c0 + j]; is[j] = invstd[c0 + j];
    sg[j] = 0.f; sgx[j] = 0.f;
  }
  // four voxel rows' loads in flight per trip, accumulated in the same voxel order as one
  // at a time (identical sums)
  const long stride = (long)gridDim.x * VL;
  long v = (long)blockIdx.x * VL + vl;
  auto acc1 = [&](const float (&dv)[VEC], const float (&yv)[VEC]) {
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      const float g = (yv[j] * sc[j] + sh[j] > 0.f) ? dv[j] : 0.f;
      sg[j] += g;
      sgx[j] += g * ((yv[j] - mu[j]) * is[j]);
    }
  };
#ifndef BNR_U
#define BNR_U 2  // voxel rows in flight per thread and trip (A/B: 1 / 4 / 8 slower, profiles/r4_bnr_unroll_ab.txt)
#endif
  for (; v + (BNR_U - 1) * stride < nvox; v += BNR_U * stride) {
    float dv[BNR_U][VEC], yv[BNR_U][VEC];
#pragma unroll
    for (int u = 0; u < BNR_U; ++u) {
      ld16<NT>(da + (v + u * stride) * C + c0, dv[u]);
      ld16<NT>(y + (v + u * stride) * C + c0, yv[u]);
    }
#pragma unroll
    for (int u = 0; u < BNR_U; ++u) acc1(dv[u], yv[u]);
  }
  for (; v < nvox; v += stride) {
    float dv[VEC], yv[VEC];
    load16<T>(da + v * C + c0, dv);
    load16<T>(y + v * C + c0, yv);
    acc1(dv, yv);
  }
#pragma unroll
  for (int j = 0; j < VEC; ++j) {
    red[(vl * C + c0 + j) * 2] = sg[j];
    red[(vl * C + c0 + j) * 2 + 1] = sgx[j];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += TPB) {
    float a = 0.f, b = 0.f;
    for (int l = 0; l < VL; ++l) { a += red[(l * C + c) * 2]; b += red[(l * C + c) * 2 + 1]; }
    part[((long)blockIdx.x * C + c) * 2] = a;
    part[((long)blockIdx.x * C + c) * 2 + 1] = b;
  }
}

// pass 2: fp64 column sums -> dgamma/dbeta (+=) and the apply coefficients
//   dy = k1*g + k2*xhat + k3, k1 = gamma*invstd, k2 = -k1*sum(g xhat)/M, k3 = -k1*sum(g)/M
__device__ __forceinline__ void bn_bwd_finalize_one(int c, double s1, double s2, double count, const float* gamma,
                                                    const float* invstd, float* dgamma, float* dbeta, float* coef) {
  dbeta[c] += (float)s1;
  dgamma[c] += (float)s2;
  const double k1 = (double)gamma[c] * (double)invstd[c];
  coef[c * 3 + 0] = (float)k1;
  coef[c * 3 + 1] = (float)(-k1 * s2 / count);
  coef[c * 3 + 2] = (float)(-k1 * s1 / count);
}
__global__ void bn_bwd_finalize_kernel(const double* ws, int C, double count, const float* gamma,
                                       const float* invstd, float* dgamma, float* dbeta, float* coef) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double s1, s2;
  colsum_final(ws, C, c, s1, s2);
  bn_bwd_finalize_one(c, s1, s2, count, gamma, invstd, dgamma, dbeta, coef);
}

// Few partial rows (<= kSmallRows): the column sums and the finalize in ONE launch, one block
// per 64 channels (no cross-block dependency): 4 row lanes x 64 channels, lane rl adds rows
// rl, rl + 4, ... in order (8 rows' loads in flight), the 4 lanes summed in a fixed order
// (deterministic).  Saves the second launch of the two-stage path (~5 us each, 36 per step).
constexpr int kSmallRows = 512;
// 16 row lanes x 64 channels per block: a thread sums every 16th partial row, 8 rows' loads
// in flight per trip (the sums were latency-bound chains of ~rows / 32 dependent trips on 4
// row lanes); the 16 lane sums are added in lane order
constexpr int kCfRL = 16;
// rows in flight per thread per trip (16: one trip for <= 256 rows, two for 512; 8 took up to
// four dependent trips of memory latency); the row order of every sum is the same for any value
#ifndef PCMS_CF_U
#define PCMS_CF_U 16
#endif
constexpr int kCfU = PCMS_CF_U;
template <bool BWD>
__global__ void __launch_bounds__(64 * kCfRL) colsum_finalize_small_kernel(
    const float* part, int rows, int C, const float* cnt, double count, const float* gamma, const float* beta,
    float* rmean, float* rvar, long long* nbt, float momentum, float eps, float* scale, float* shift,
    float* mean_out, float* invstd, float* dgamma, float* dbeta, float* coef) {
  __shared__ double red[kCfRL][64][2];
  const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  if (!BWD && nbt && blockIdx.x == 0 && threadIdx.x == 0) *nbt += 1;
  double s1 = 0.0, s2 = 0.0;
  if (c < C) {
    int r = rl;
    for (; r < rows; r += kCfU * kCfRL) {  // the last trip predicated, loads still batched
      float2 v[kCfU];
      float nv[kCfU];
#pragma unroll
      for (int u = 0; u < kCfU; ++u)
        if (r + kCfRL * u < rows) {
          v[u] = *reinterpret_cast<const float2*>(part + ((long)(r + kCfRL * u) * C + c) * 2);
          nv[u] = cnt ? cnt[r + kCfRL * u] : 0.f;
        }
#pragma unroll
      for (int u = 0; u < kCfU; ++u) {
        if (r + kCfRL * u >= rows) break;
        s1 += (double)v[u].x;
        if (cnt) {
          const double n = (double)nv[u];
          s2 += (double)v[u].y + (n > 0.0 ? (double)v[u].x * (double)v[u].x / n : 0.0);
        } else {
          s2 += (double)v[u].y;
        }
      }
    }
  }
  red[rl][cl][0] = s1;
  red[rl][cl][1] = s2;
  __syncthreads();
  if (rl == 0 && c < C) {
    for (int g = 1; g < kCfRL; ++g) { s1 += red[g][cl][0]; s2 += red[g][cl][1]; }
    if constexpr (BWD) bn_bwd_finalize_one(c, s1, s2, count, gamma, invstd, dgamma, dbeta, coef);
    else bn_finalize_one(c, s1, s2, count, gamma, beta, rmean, rvar, momentum, eps, scale, shift, mean_out, invstd);
  }
}

#ifndef BNA_REV
#define BNA_REV 0
#endif
// BatchNorm + ReLU backward of one element, dy = k1 g + k2 xhat + k3 with g = da [y sc + sh > 0]:
// the operations written out (fma(y, sc, sh) for the mask, fma(k2, xhat, k1 g) + k3) so that
// every kernel applying it rounds the same way -- the compiler's own contraction of the plain
// expression picked fma(k1, g, k2 xhat) in one kernel and fma(k2, xhat, k1 g) in another
__device__ __forceinline__ float bn_bwd_dy(float da, float y, float sc, float sh, float mu, float is, float k1,
                                           float k2, float k3) {
#pragma clang fp contract(off)
  const float g = __builtin_fmaf(y, sc, sh) > 0.f ? da : 0.f;
  const float xhat = (y - mu) * is;
  return __builtin_fmaf(k2, xhat, k1 * g) + k3;
}
// NT: as bn_relu_kernel (level-0 apply: 805 MB in 118 us = 6.8 TB/s)
template <typename T, bool NT>
__global__ void __launch_bounds__(TPB) bn_relu_bwd_apply_kernel(
    const T* da, const T* y, const float* scale, const float* shift, const float* mean, const float* invstd,
    const float* coef, T* dy, int C, long nvox) {
  constexpr int VEC = Elem<T>::kVec;
  const int CG = C / VEC;
  const int cg = threadIdx.x % CG, vl = threadIdx.x / CG, VL = TPB / CG;
  const int c0 = cg * VEC;
  float sc[VEC], sh[VEC], mu[VEC], is[VEC], k1[VEC], k2[VEC], k3[VEC];
#pragma unroll
  for (int j = 0; j < VEC; ++j) {
    const int c = c0 + j;
    sc[j] = scale[c]; sh[j] = shift[c]; mu[j] = mean[c]; is[j] = invstd[c];
    k1[j] = coef[c * 3]; k2[j] = coef[c * 3 + 1]; k3[j] = coef[c * 3 + 2];
  }
  for (long v0 = (long)blockIdx.x * VL + vl; v0 < nvox; v0 += (long)gridDim.x * VL) {
    // BNA_REV: walk the voxels from the end -- the reduce pass before this one finishes at the
    // high voxels, so what it left in the Infinity Cache is read first (elementwise: any order
    // gives the same bits)
    const long v = BNA_REV ? nvox - 1 - v0 : v0;
    float dv[VEC], yv[VEC], o[VEC];
    ld16<NT>(da + v * C + c0, dv);
    ld16<NT>(y + v * C + c0, yv);
#pragma unroll
    for (int j = 0; j < VEC; ++j) o[j] = bn_bwd_dy(dv[j], yv[j], sc[j], sh[j], mu[j], is[j], k1[j], k2[j], k3[j]);
    st16<NT>(dy + v * C + c0, o);
  }
}

// ---------------- MaxPool3d(2), floor mode; first max wins (PyTorch scan order) -------
template <typename T>
__global__ void maxpool_fwd_kernel(const T* a, T* p, int N, int D, int H, int W, int C) {
  constexpr int VEC = Elem<T>::kVec;
  const int Do = D / 2, Ho = H / 2, Wo = W / 2, CV = C / VEC;
  const long total = (long)N * Do * Ho * Wo * CV;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    // 32-bit index decomposition (host: total < 2^31): 64-bit division is a long sequence
    const uint32_t ii = (uint32_t)i;
    const int cv = ii % CV; uint32_t r = ii / CV;
    const int wo = r % Wo; r /= Wo;
    const int ho = r % Ho; r /= Ho;
    const int d_o = r % Do; const long n = r / Do;
    float m[VEC];
#pragma unroll
    for (int j = 0; j < VEC; ++j) m[j] = -INFINITY;
    for (int k = 0; k < 8; ++k) {
      const long vin = ((n * D + 2 * d_o + (k >> 2)) * H + 2 * ho + ((k >> 1) & 1)) * W + 2 * wo + (k & 1);
      float v[VEC];
      load16<T>(a + vin * C + cv * VEC, v);
#pragma unroll
      for (int j = 0; j < VEC; ++j)
        if (v[j] > m[j] || v[j] != v[j]) m[j] = v[j];
    }
    store16<T>(p + i * VEC, m);
  }
}

// da[argmax] += dp (da already holds the skip-path gradient)
template <typename T>
__global__ void maxpool_bwd_kernel(const T* a, const T* dp, T* da, int N, int D, int H, int W, int C) {
  constexpr int VEC = Elem<T>::kVec;
  const int Do = D / 2, Ho = H / 2, Wo = W / 2, CV = C / VEC;
  const long total = (long)N * Do * Ho * Wo * CV;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const uint32_t ii = (uint32_t)i;  // 32-bit index decomposition (host: total < 2^31)
    const int cv = ii % CV; uint32_t r = ii / CV;
    const int wo = r % Wo; r /= Wo;
    const int ho = r % Ho; r /= Ho;
    const int d_o = r % Do; const long n = r / Do;
    float m[VEC];
    int arg[VEC];
#pragma unroll
    for (int j = 0; j < VEC; ++j) { m[j] = -INFINITY; arg[j] = 0; }
    long vin[8];
    for (int k = 0; k < 8; ++k) {
      vin[k] = ((n * D + 2 * d_o + (k >> 2)) * H + 2 * ho + ((k >> 1) & 1)) * W + 2 * wo + (k & 1);
      float v[VEC];
      load16<T>(a + vin[k] * C + cv * VEC, v);
#pragma unroll
      for (int j = 0; j < VEC; ++j)
        if (v[j] > m[j] || (v[j] != v[j] && m[j] == m[j])) { m[j] = v[j]; arg[j] = k; }
    }
    float g[VEC];
    load16<T>(dp + i * VEC, g);
    for (int k = 0; k < 8; ++k) {
      float o[VEC];
      load16<T>(da + vin[k] * C + cv * VEC, o);
#pragma unroll
      for (int j = 0; j < VEC; ++j) o[j] += (arg[j] == k) ? g[j] : 0.f;
      store16<T>(da + vin[k] * C + cv * VEC, o);
    }
  }
}

// ---------------- encoder block output: BN + ReLU fused with the MaxPool3d of Down3D --------
// (models/unet3d.py:37-39 of a DoubleConv, then :80 of the next Down3D.)  One thread per
// (2x2x2 cell of the ceil-sized grid, VEC channels): a = round_T(relu(y sc + sh)) for the cell's
// children is stored (the block output, read by the skip connection), and for whole cells the
// max of those stored values (maxpool_fwd_kernel's scan order and NaN rule) -- the output is
// pooled while it is in registers instead of being read back by a separate pass.
template <typename T, bool NT>
__global__ void __launch_bounds__(TPB) bn_relu_pool_kernel(const T* y, T* a, T* p, const float* scale,
                                                           const float* shift, int N, int D, int H, int W,
                                                           int C) {
  constexpr int VEC = Elem<T>::kVec;
  const int Dc = (D + 1) / 2, Hc = (H + 1) / 2, Wc = (W + 1) / 2, CV = C / VEC;
  const int Do = D / 2, Ho = H / 2, Wo = W / 2;
  const long total = (long)N * Dc * Hc * Wc * CV;
  const long stride = (long)gridDim.x * blockDim.x;  // multiple of CV (host): cv is per thread
  long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  const int cv = (int)(i % CV);
  float sc[VEC], sh[VEC];
#pragma unroll
  for (int j = 0; j < VEC; ++j) { sc[j] = scale[cv * VEC + j]; sh[j] = shift[cv * VEC + j]; }
  for (; i < total; i += stride) {
    uint32_t r = (uint32_t)(i / CV);  // 32-bit decomposition (host: cells < 2^31)
    const int wc = r % Wc; r /= Wc;
    const int hc = r % Hc; r /= Hc;
    const int dc = r % Dc; const long n = r / Dc;
    float m[VEC];
#pragma unroll
    for (int j = 0; j < VEC; ++j) m[j] = -INFINITY;
    float v[8][VEC];
    long vin[8];
    bool in[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int d = 2 * dc + (k >> 2), h = 2 * hc + ((k >> 1) & 1), w = 2 * wc + (k & 1);
      in[k] = d < D && h < H && w < W;
      vin[k] = ((n * D + d) * H + h) * W + w;
#ifndef BRP_NTLOAD
#define BRP_NTLOAD 1  // A/B: y loads non-temporal with the stores (1) or cached (0)
#endif
      if (in[k]) ld16<NT && BRP_NTLOAD>(y + vin[k] * C + cv * VEC, v[k]);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (!in[k]) continue;
#pragma unroll
      for (int j = 0; j < VEC; ++j) v[k][j] = round_st<T>(bn_relu1(v[k][j], sc[j], sh[j]));
      st16<NT>(a + vin[k] * C + cv * VEC, v[k]);
#pragma unroll
      for (int j = 0; j < VEC; ++j)
        if (v[k][j] > m[j] || v[k][j] != v[k][j]) m[j] = v[k][j];
    }
    if (dc < Do && hc < Ho && wc < Wo) store16<T>(p + (((n * Do + dc) * Ho + hc) * Wo + wc) * C + cv * VEC, m);
  }
}

// MaxPool3d backward fused with the BatchNorm + ReLU backward reduction of the block whose
// output was pooled: da (the block output's gradient, already holding the skip-path part) +=
// dp at the argmax of a = round_T(relu(y sc + sh)) -- a recomputed from y exactly as
// bn_relu_pool_kernel stored it, maxpool_bwd_kernel's first-max / NaN rule -- and, over every
// voxel (the floor-mode leftovers too), the partial sums of g = da [y sc + sh > 0] and g xhat
// per channel: one [C][2] row per block (bn_relu_bwd_reduce_kernel's quantities), so the
// BatchNorm backward needs no reduction pass over da and y of its own.
// STORE false (pcms_maxpool_bwd_bn_sums): the same sums, da left as it was (the skip-path part
// only) -- maxpool_bn_apply_kernel forms the pooled-path sum again where it applies the BN.
template <typename T, bool STORE = true>
__global__ void __launch_bounds__(TPB, 3) maxpool_bwd_bn_kernel(const T* y, const float* scale, const float* shift,
                                                             const float* mean, const float* invstd, const T* dp,
                                                             T* da, float* part, int N, int D, int H, int W,
                                                             int C) {
  constexpr int VEC = Elem<T>::kVec;
  __shared__ float red[TPB][VEC][2];
  const int Dc = (D + 1) / 2, Hc = (H + 1) / 2, Wc = (W + 1) / 2, CV = C / VEC;
  const int Do = D / 2, Ho = H / 2, Wo = W / 2;
  const long total = (long)N * Dc * Hc * Wc * CV;
  const long stride = (long)gridDim.x * blockDim.x;  // multiple of CV (host)
  long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  const int cv = (int)(i % CV);
  float sc[VEC], sh[VEC], mu[VEC], is[VEC], sg[VEC], sgx[VEC];
#pragma unroll
  for (int j = 0; j < VEC; ++j) {
    const int c = cv * VEC + j;
    sc[j] = scale[c]; sh[j] = shift[c]; mu[j] = mean[c]; is[j] = invstd[c];
    sg[j] = 0.f; sgx[j] = 0.f;
  }
  // a cell's 8 y chunks, 8 da chunks and its dp chunk are all loaded (raw 16-B vectors) before
  // the first use: one memory round trip per cell instead of one per child
  auto unpack = [](const u32x4_t r, float (&o)[VEC]) {
    if constexpr (sizeof(T) == 2) {
#pragma unroll
      for (int q = 0; q < 4; ++q) { o[2 * q] = __uint_as_float(r[q] << 16); o[2 * q + 1] = __uint_as_float(r[q] & 0xffff0000u); }
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) o[q] = __uint_as_float(r[q]);
    }
  };
  for (; i < total; i += stride) {
    uint32_t r = (uint32_t)(i / CV);
    const int wc = r % Wc; r /= Wc;
    const int hc = r % Hc; r /= Hc;
    const int dc = r % Dc; const long n = r / Dc;
    const bool whole = dc < Do && hc < Ho && wc < Wo;
    u32x4_t yr[8], dr[8], gr = {0u, 0u, 0u, 0u};
    // child k: voxel v0 + (k >> 2) H W + ((k >> 1) & 1) W + (k & 1) (recomputed where used)
    const long v0 = ((n * D + 2 * dc) * H + 2 * hc) * W + 2 * wc;
    const bool ind = 2 * dc + 1 < D, inh = 2 * hc + 1 < H, inw = 2 * wc + 1 < W;
    auto vk = [&](int k) { return v0 + (long)(k >> 2) * H * W + ((k >> 1) & 1) * W + (k & 1); };
    auto ink = [&](int k) { return (!(k & 4) || ind) && (!(k & 2) || inh) && (!(k & 1) || inw); };
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      yr[k] = (u32x4_t){0u, 0u, 0u, 0u};
      dr[k] = yr[k];
      if (ink(k)) {
        yr[k] = *reinterpret_cast<const u32x4_t*>(y + vk(k) * C + cv * VEC);
        dr[k] = *reinterpret_cast<const u32x4_t*>(da + vk(k) * C + cv * VEC);
      }
    }
    if (whole) gr = *reinterpret_cast<const u32x4_t*>(dp + (((n * Do + dc) * Ho + hc) * Wo + wc) * C + cv * VEC);
    float g[VEC], m[VEC];
    int arg[VEC];
    unpack(gr, g);
#pragma unroll
    for (int j = 0; j < VEC; ++j) { m[j] = -INFINITY; arg[j] = 0; }
    // channel pairs in packed fp32 (the same IEEE operation per element as the scalar forms,
    // half the VALU issue: the kernel was VALU-bound) and one v_cvt_pk_bf16_f32 per pair
    auto round2 = [](f32x2_t v) -> f32x2_t {
      if constexpr (sizeof(T) == 2) {
        const uint32_t u = pack_bf16x2(v[0], v[1]);
        return (f32x2_t){__uint_as_float(u << 16), __uint_as_float(u & 0xffff0000u)};
      } else {
        return v;
      }
    };
    auto z2of = [&](const float (&yv)[VEC], int q) {
      return __builtin_elementwise_fma((f32x2_t){yv[2 * q], yv[2 * q + 1]}, (f32x2_t){sc[2 * q], sc[2 * q + 1]},
                                       (f32x2_t){sh[2 * q], sh[2 * q + 1]});
    };
    if (whole) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float yv[VEC];
        unpack(yr[k], yv);
#pragma unroll
        for (int j = 0; j < VEC; ++j) {
          const float av = round_st<T>(bn_relu1(yv[j], sc[j], sh[j]));
          if (av > m[j] || (av != av && m[j] == m[j])) { m[j] = av; arg[j] = k; }
        }
      }
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (!ink(k)) continue;
      float yv[VEC], o[VEC];
      // (an opaque copy: the compiler would otherwise keep the argmax pass's 64 BN values live
      // for this pass, past the register budget)
      u32x4_t yk = yr[k];
      asm volatile("" : "+v"(yk));
      unpack(yk, yv);
      unpack(dr[k], o);
      if (whole) {
#pragma unroll
        for (int j = 0; j < VEC; ++j) o[j] += (arg[j] == k) ? g[j] : 0.f;
        if constexpr (STORE) store16<T>(da + vk(k) * C + cv * VEC, o);
      }
#pragma unroll
      for (int q = 0; q < VEC / 2; ++q) {
        const f32x2_t z2 = z2of(yv, q);
        const f32x2_t r2 = round2((f32x2_t){o[2 * q], o[2 * q + 1]});
        const f32x2_t g2 = {z2[0] > 0.f ? r2[0] : 0.f, z2[1] > 0.f ? r2[1] : 0.f};
        const f32x2_t t2 = ((f32x2_t){yv[2 * q], yv[2 * q + 1]} - (f32x2_t){mu[2 * q], mu[2 * q + 1]}) *
                           (f32x2_t){is[2 * q], is[2 * q + 1]};
        f32x2_t sg2 = {sg[2 * q], sg[2 * q + 1]}, sgx2 = {sgx[2 * q], sgx[2 * q + 1]};
        {
#pragma clang fp contract(off)  // a product then a sum, as the separate reduce pass forms it
          sgx2 = sgx2 + g2 * t2;
          sg2 = sg2 + g2;
        }
        sg[2 * q] = sg2[0]; sg[2 * q + 1] = sg2[1];
        sgx[2 * q] = sgx2[0]; sgx[2 * q + 1] = sgx2[1];
      }
    }
  }
#pragma unroll
  for (int j = 0; j < VEC; ++j) { red[threadIdx.x][j][0] = sg[j]; red[threadIdx.x][j][1] = sgx[j]; }
  __syncthreads();
  // this block's row: channel c = cv' VEC + j sums threads t = cv' + CV k in t order
  const int c0 = (int)(((long)blockIdx.x * blockDim.x) % CV);  // the cv of thread 0
  for (int e = threadIdx.x; e < C * 2; e += TPB) {
    const int c = e >> 1, q = e & 1, cvc = c / VEC, j = c % VEC;
    const int t0 = (cvc - c0 + CV) % CV;
    float acc = 0.f;
    for (int t = t0; t < TPB; t += CV) acc += red[t][j][q];
    part[((long)blockIdx.x * C + c) * 2 + q] = acc;
  }
}

// The consumer half of the pair above (pcms_maxpool_bn_apply): per 2x2x2 cell, the block
// output's gradient da = gx + dp at the argmax -- recomputed from y exactly as
// maxpool_bwd_bn_kernel forms it, rounded to T as that kernel stores it -- and then
// bn_relu_bwd_apply_kernel's dy = k1 g + k2 xhat + k3 (its arithmetic, expression for
// expression).  With pcms_maxpool_bwd_bn_sums before it, da is never written to HBM: this
// pass reads gx + dp (+ 1/8 of a tensor) where the stored form wrote da and read it back.
template <typename T, bool NT>
// (two blocks per CU: its 7 x VEC per-channel coefficients do not fit the three-block budget)
__global__ void __launch_bounds__(TPB, 2) maxpool_bn_apply_kernel(const T* y, const float* scale, const float* shift,
                                                               const float* mean, const float* invstd,
                                                               const float* coef, const T* dp, const T* gx, T* dy,
                                                               int N, int D, int H, int W, int C) {
  constexpr int VEC = Elem<T>::kVec;
  const int Dc = (D + 1) / 2, Hc = (H + 1) / 2, Wc = (W + 1) / 2, CV = C / VEC;
  const int Do = D / 2, Ho = H / 2, Wo = W / 2;
  const long total = (long)N * Dc * Hc * Wc * CV;
  const long stride = (long)gridDim.x * blockDim.x;  // multiple of CV (host)
  long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  const int cv = (int)(i % CV);
  float sc[VEC], sh[VEC], mu[VEC], is[VEC], k1[VEC], k2[VEC], k3[VEC];
#pragma unroll
  for (int j = 0; j < VEC; ++j) {
    const int c = cv * VEC + j;
    sc[j] = scale[c]; sh[j] = shift[c]; mu[j] = mean[c]; is[j] = invstd[c];
    k1[j] = coef[c * 3]; k2[j] = coef[c * 3 + 1]; k3[j] = coef[c * 3 + 2];
  }
  for (; i < total; i += stride) {
    uint32_t r = (uint32_t)(i / CV);
    const int wc = r % Wc; r /= Wc;
    const int hc = r % Hc; r /= Hc;
    const int dc = r % Dc; const long n = r / Dc;
    const bool whole = dc < Do && hc < Ho && wc < Wo;
    const long v0 = ((n * D + 2 * dc) * H + 2 * hc) * W + 2 * wc;
    const bool ind = 2 * dc + 1 < D, inh = 2 * hc + 1 < H, inw = 2 * wc + 1 < W;
    auto vk = [&](int k) { return v0 + (long)(k >> 2) * H * W + ((k >> 1) & 1) * W + (k & 1); };
    auto ink = [&](int k) { return (!(k & 4) || ind) && (!(k & 2) || inh) && (!(k & 1) || inw); };
    // raw 16-B vectors (4 registers each), unpacked where used: the cell's 16 loads and its
    // dp load all in flight before the first use, in maxpool_bwd_bn_kernel's register budget
    auto unpack = [](const u32x4_t r, float (&o)[VEC]) {
      if constexpr (sizeof(T) == 2) {
#pragma unroll
        for (int q = 0; q < 4; ++q) { o[2 * q] = __uint_as_float(r[q] << 16); o[2 * q + 1] = __uint_as_float(r[q] & 0xffff0000u); }
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) o[q] = __uint_as_float(r[q]);
      }
    };
    auto ldraw = [](const T* p) -> u32x4_t {
      if constexpr (NT) return __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(p));
      else return *reinterpret_cast<const u32x4_t*>(p);
    };
    u32x4_t yr[8], dr[8], gr = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      yr[k] = (u32x4_t){0u, 0u, 0u, 0u};
      dr[k] = yr[k];
      if (ink(k)) {
        yr[k] = ldraw(y + vk(k) * C + cv * VEC);
        dr[k] = ldraw(gx + vk(k) * C + cv * VEC);
      }
    }
    if (whole) gr = *reinterpret_cast<const u32x4_t*>(dp + (((n * Do + dc) * Ho + hc) * Wo + wc) * C + cv * VEC);
    float g[VEC], m[VEC];
    int arg[VEC];
    unpack(gr, g);
#pragma unroll
    for (int j = 0; j < VEC; ++j) { m[j] = -INFINITY; arg[j] = 0; }
    if (whole) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float yv[VEC];
        unpack(yr[k], yv);
#pragma unroll
        for (int j = 0; j < VEC; ++j) {
          const float av = round_st<T>(bn_relu1(yv[j], sc[j], sh[j]));
          if (av > m[j] || (av != av && m[j] == m[j])) { m[j] = av; arg[j] = k; }
        }
      }
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (!ink(k)) continue;
      float yv[VEC], o[VEC], out[VEC];
      u32x4_t yk = yr[k];
      asm volatile("" : "+v"(yk));  // (as maxpool_bwd_bn_kernel: keep the argmax pass's values dead)
      unpack(yk, yv);
      unpack(dr[k], o);
      if (whole) {
#pragma unroll
        for (int j = 0; j < VEC; ++j) o[j] = round_st<T>(o[j] + ((arg[j] == k) ? g[j] : 0.f));
      }
#pragma unroll
      for (int j = 0; j < VEC; ++j) out[j] = bn_bwd_dy(o[j], yv[j], sc[j], sh[j], mu[j], is[j], k1[j], k2[j], k3[j]);
      st16<NT>(dy + vk(k) * C + cv * VEC, out);
    }
  }
}

// ---------------- sum over a sub-box of an NDHWC tensor (ConvT bias grad) ----------
// Block: 256 threads = (256 / CG) voxel lanes x CG groups of VEC channels; 16-byte loads,
// LDS reduce over voxel lanes, one partial row [C] per block (summed in block order by
// rows_sum_kernel: no atomics, run-to-run reproducible).
template <typename T>
__global__ void __launch_bounds__(TPB) box_channel_sum_kernel(const T* x, float* part, int N, int D, int H, int W,
                                                              int C, int z0, int y0, int x0, int bd, int bh, int bw) {
  constexpr int VEC = Elem<T>::kVec;
  __shared__ float red[TPB * VEC];
  const int CG = C / VEC;
  const int cg = threadIdx.x % CG, vl = threadIdx.x / CG, VL = TPB / CG;
  const long nv = (long)N * bd * bh * bw;
  float acc[VEC];
#pragma unroll
  for (int j = 0; j < VEC; ++j) acc[j] = 0.f;
  const long stride = (long)gridDim.x * VL;
  long i = (long)blockIdx.x * VL + vl;
  if (bd == D && bh == H && bw == W) {
    // the box is the whole grid (no pad): voxel i is row i; four rows' loads in flight per
    // trip, added in the same order as one at a time
    for (; i + 3 * stride < nv; i += 4 * stride) {
      float v[4][VEC];
#pragma unroll
      for (int u = 0; u < 4; ++u) load16<T>(x + (i + u * stride) * C + cg * VEC, v[u]);
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int j = 0; j < VEC; ++j) acc[j] += v[u][j];
    }
  }
  for (; i < nv; i += stride) {
    const uint32_t ii = (uint32_t)i;  // 32-bit index decomposition (host: nv < 2^31)
    const int w = ii % bw; uint32_t r = ii / bw;
    const int h = r % bh; r /= bh;
    const int d = r % bd; const long n = r / bd;
    float v[VEC];
    load16<T>(x + (((n * D + z0 + d) * H + y0 + h) * W + x0 + w) * C + cg * VEC, v);
#pragma unroll
    for (int j = 0; j < VEC; ++j) acc[j] += v[j];
  }
#pragma unroll
  for (int j = 0; j < VEC; ++j) red[vl * C + cg * VEC + j] = acc[j];
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += TPB) {
    float s = 0.f;
    for (int l = 0; l < VL; ++l) s += red[l * C + c];
    part[(long)blockIdx.x * C + c] = s;
  }
}

// out[c] += sum_r part[r][c] in a fixed order (deterministic).  Block = 8 columns x 32 row
// lanes: lane l sums rows l, l + 32, ... (4 independent chains); the 32 lane sums are
// added by a fixed LDS tree.
// ACC: out[c] += the column sum (false: out[c] = it -- no zero fill of out first)
template <bool ACC>
__global__ void __launch_bounds__(256) rows_sum_kernel(const float* part, int rows, int C, float* out) {
  __shared__ float red[32][9];
  const int cl = threadIdx.x & 7, rl = threadIdx.x >> 3;
  const int c = blockIdx.x * 8 + cl;
  float s[4] = {0.f, 0.f, 0.f, 0.f};
  if (c < C) {
    int r = rl;
    for (; r + 96 < rows; r += 128) {
#pragma unroll
      for (int j = 0; j < 4; ++j) s[j] += part[(long)(r + 32 * j) * C + c];
    }
    for (int j = 0; r < rows; r += 32, ++j) s[j & 3] += part[(long)r * C + c];
  }
  red[rl][cl] = (s[0] + s[1]) + (s[2] + s[3]);
  __syncthreads();
  for (int w = 16; w > 0; w >>= 1) {
    if (rl < w) red[rl][cl] += red[rl + w][cl];
    __syncthreads();
  }
  if (rl == 0 && c < C) out[c] = ACC ? out[c] + red[0][cl] : red[0][cl];
}

// ---------------- output head: logits (NCDHW fp32) = b + a . w ----------------
// 8 lanes per voxel, 8 channels each (Cin = 64); NC = n_classes (<= 4, a template argument
// so per-class registers exist only for real classes).  Every kernel walks kHU voxels per
// trip with all of their loads (activations and, backward, dlogits) issued before the first
// use: these are pure streams, bound by bytes in flight per CU.
constexpr int kHU = 4;

template <typename T, bool NT>
__device__ __forceinline__ void head_ld(const T* p, float (&x)[8]) {
  ld16<NT>(p, x);
  if constexpr (sizeof(T) == 4) ld16<NT>(p + 4, x + 4);
}
template <typename T, bool NT>
__device__ __forceinline__ void head_st(T* p, const float (&x)[8]) {
  st16<NT>(p, x);
  if constexpr (sizeof(T) == 4) st16<NT>(p + 4, x + 4);
}

// act 0: logits; 1: sigmoid(logits) (UNet3D.predict, models/unet3d.py:298-318); 2:
// (sigmoid(logits) > thr) as 0 / 1 (UNet3D.inference, :320-344) -- the eval outputs leave the
// head kernel finished.
// BN: ``a`` is the decoder's last pre-BN conv output y2 and the head applies that block's
// BatchNorm + ReLU itself (models/unet3d.py:37-39 fused into :222): a = round_T(relu(y sc +
// sh)), the value the bn_relu pass would have stored, so the logits are bit-identical and
// the a2 tensor (the largest activation of the step) is never written or read.
// voxel v of an (N, nvox) grid as (sample q, voxel-in-sample r), stepped without a division
// per voxel (the heads index the NCDHW logit gradient by both; a runtime 32-bit division per
// lane and voxel was a large share of their VALU)
struct VoxQR {
  uint32_t q, r, nv;
  __device__ VoxQR(long v, long nvox) : q((uint32_t)(v / nvox)), r((uint32_t)(v % nvox)), nv((uint32_t)nvox) {}
  __device__ void advance(uint32_t k) {
    r += k;
    while (r >= nv) { r -= nv; ++q; }
  }
  __device__ VoxQR plus(uint32_t k) const {
    VoxQR o = *this;
    o.advance(k);
    return o;
  }
};

template <typename T, bool NT, bool BN, int NC>
__global__ void __launch_bounds__(TPB, 3) head_fwd_kernel(const T* a, const float* w, const float* b, float* logits,
                                                       long nvox_per_n, int N, int act, float thr,
                                                       const float* bn_scale, const float* bn_shift) {
  const long total = (long)N * nvox_per_n;
  const int sub = threadIdx.x & 7;
  float sc[8], sh[8], wk[NC][8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    if constexpr (BN) { sc[j] = bn_scale[sub * 8 + j]; sh[j] = bn_shift[sub * 8 + j]; }
#pragma unroll
    for (int k = 0; k < NC; ++k) wk[k][j] = w[k * 64 + sub * 8 + j];
  }
  auto one = [&](const VoxQR& p, float (&x)[8]) {
    if constexpr (BN) {
#pragma unroll
      for (int j = 0; j < 8; ++j) x[j] = round_st<T>(bn_relu1(x[j], sc[j], sh[j]));
    }
#pragma unroll
    for (int k = 0; k < NC; ++k) {
      float s = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) s += x[j] * wk[k][j];
      s += __shfl_xor(s, 1, 64);
      s += __shfl_xor(s, 2, 64);
      s += __shfl_xor(s, 4, 64);
      if (sub == 0) {
        float o = s + b[k];
        if (act != 0) {
          const float pr = 1.f / (1.f + expf(-o));
          o = act == 1 ? pr : (pr > thr ? 1.f : 0.f);
        }
        logits[((long)p.q * NC + k) * nvox_per_n + p.r] = o;
      }
    }
  };
  const long stride = ((long)gridDim.x * blockDim.x) >> 3;
  long v = (blockIdx.x * (long)blockDim.x + threadIdx.x) >> 3;
  VoxQR pv(v, nvox_per_n);
  for (; v + (kHU - 1) * stride < total; v += kHU * stride) {
    float x[kHU][8];
#pragma unroll
    for (int u = 0; u < kHU; ++u) head_ld<T, NT>(a + (v + u * stride) * 64 + sub * 8, x[u]);
#pragma unroll
    for (int u = 0; u < kHU; ++u) one(u ? pv.plus((uint32_t)(u * stride)) : pv, x[u]);
    pv.advance((uint32_t)(kHU * stride));
  }
  for (; v < total; v += stride) {
    float x[8];
    head_ld<T, NT>(a + v * 64 + sub * 8, x);
    one(pv, x);
    pv.advance((uint32_t)stride);
  }
}

// da[v, c] = sum_k dl[k, v] w[k, c]  (written);  per-block partials of dw[k, c] = sum_v dl a,
// db[k] = sum_v dl.  NT: non-temporal a / da streams (level-0 sized).
// BN (the decoder's last BatchNorm + ReLU fused, see head_fwd_kernel): ``a`` is y2; the head
// input a2 = round_T(relu(y sc + sh)) is recomputed, da is NOT written: its round_T value
// feeds the BatchNorm-backward partial sums directly -- per block one row [64][2] of
// (sum g, sum g xhat), g = da [y sc + sh > 0], xhat = (y - mean) invstd -- and
// head_bn_apply_kernel recomputes da from dlogits (rank NC) instead of re-reading it.
struct HeadBN {
  const float *scale, *shift, *mean, *invstd;
  float* part;  // [blocks][64][2]
};
template <typename T, bool NT, bool BN, int NC>
__global__ void __launch_bounds__(TPB, (BN && NC > 2) ? 2 : 3) head_bwd_kernel(const T* a, const float* dlogits, const float* w,
                                                       T* da, float* part, long nvox_per_n, int N, HeadBN bn) {
  __shared__ float red[TPB / 64][NC][65];
  __shared__ float bred[TPB / 64][64][2];
  const long total = (long)N * nvox_per_n;
  const int sub = threadIdx.x & 7, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float accw[NC][8], accb[NC], wk[NC][8];
  float sc[8], sh[8], mu[8], is[8], sg[8], sgx[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
#pragma unroll
    for (int k = 0; k < NC; ++k) { accw[k][j] = 0.f; wk[k][j] = w[k * 64 + sub * 8 + j]; }
    if constexpr (BN) {
      const int c = sub * 8 + j;
      sc[j] = bn.scale[c]; sh[j] = bn.shift[c]; mu[j] = bn.mean[c]; is[j] = bn.invstd[c];
      sg[j] = 0.f; sgx[j] = 0.f;
    }
  }
#pragma unroll
  for (int k = 0; k < NC; ++k) accb[k] = 0.f;
  auto ld_dl = [&](const VoxQR& p, float (&dl)[NC]) {
#pragma unroll
    for (int k = 0; k < NC; ++k) dl[k] = dlogits[((long)p.q * NC + k) * nvox_per_n + p.r];
  };
  // channel pairs in packed fp32 (v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32: the same IEEE
  // operation per element as the scalar forms, half the VALU issue; the kernel was VALU-bound)
  // and one v_cvt_pk_bf16_f32 per pair for the T rounding
  auto round2 = [](f32x2_t v) -> f32x2_t {
    if constexpr (sizeof(T) == 2) {
      const uint32_t u = pack_bf16x2(v[0], v[1]);
      return (f32x2_t){__uint_as_float(u << 16), __uint_as_float(u & 0xffff0000u)};
    } else {
      return v;
    }
  };
  auto one = [&](long v, const float (&x)[8], const float (&dl)[NC]) {
    float o[8];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const f32x2_t x2 = {x[2 * q], x[2 * q + 1]};
      f32x2_t z2 = {0.f, 0.f}, av2 = x2;
      if constexpr (BN) {
        z2 = __builtin_elementwise_fma(x2, (f32x2_t){sc[2 * q], sc[2 * q + 1]}, (f32x2_t){sh[2 * q], sh[2 * q + 1]});
        av2 = round2((f32x2_t){fmaxf(z2[0], 0.f), fmaxf(z2[1], 0.f)});
      }
      f32x2_t o2 = {0.f, 0.f};
#pragma unroll
      for (int k = 0; k < NC; ++k) {
        const f32x2_t d2 = {dl[k], dl[k]};
        o2 = __builtin_elementwise_fma(d2, (f32x2_t){wk[k][2 * q], wk[k][2 * q + 1]}, o2);
        const f32x2_t a2 = __builtin_elementwise_fma(d2, av2, (f32x2_t){accw[k][2 * q], accw[k][2 * q + 1]});
        accw[k][2 * q] = a2[0];
        accw[k][2 * q + 1] = a2[1];
      }
      if constexpr (BN) {
        const f32x2_t r2 = round2(o2);
        const f32x2_t g2 = {z2[0] > 0.f ? r2[0] : 0.f, z2[1] > 0.f ? r2[1] : 0.f};
        const f32x2_t t2 = (x2 - (f32x2_t){mu[2 * q], mu[2 * q + 1]}) * (f32x2_t){is[2 * q], is[2 * q + 1]};
        // sum g xhat as a product then a sum (not fused), as the separate reduce pass forms it
        f32x2_t sgx2 = {sgx[2 * q], sgx[2 * q + 1]}, sg2 = {sg[2 * q], sg[2 * q + 1]};
        {
#pragma clang fp contract(off)
          sgx2 = sgx2 + g2 * t2;
          sg2 = sg2 + g2;
        }
        sg[2 * q] = sg2[0]; sg[2 * q + 1] = sg2[1];
        sgx[2 * q] = sgx2[0]; sgx[2 * q + 1] = sgx2[1];
      }
      o[2 * q] = o2[0];
      o[2 * q + 1] = o2[1];
    }
#pragma unroll
    for (int k = 0; k < NC; ++k)
      if (sub == 0) accb[k] += dl[k];
    if constexpr (!BN) head_st<T, NT>(da + v * 64 + sub * 8, o);
  };
  const long stride = ((long)gridDim.x * blockDim.x) >> 3;
  long v = (blockIdx.x * (long)blockDim.x + threadIdx.x) >> 3;
  VoxQR pv(v, nvox_per_n);
#ifndef HEADB_U
#define HEADB_U 2
#endif
  constexpr int U = NC > 2 ? 1 : (BN || NC > 1) ? HEADB_U : kHU;  // (registers: the BN form holds 6 x 8 per-channel values)
#pragma unroll 1
  for (; v + (U - 1) * stride < total; v += U * stride) {
    float x[U][8], dl[U][NC];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      head_ld<T, NT>(a + (v + u * stride) * 64 + sub * 8, x[u]);
      ld_dl(u ? pv.plus((uint32_t)(u * stride)) : pv, dl[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) one(v + u * stride, x[u], dl[u]);
    pv.advance((uint32_t)(U * stride));
  }
  for (; v < total; v += stride) {
    float x[8], dl[NC];
    head_ld<T, NT>(a + v * 64 + sub * 8, x);
    ld_dl(pv, dl);
    one(v, x, dl);
    pv.advance((uint32_t)stride);
  }
  // reduce accw over the 8 voxel-lanes of each wave that share `sub`
#pragma unroll
  for (int k = 0; k < NC; ++k) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float s = accw[k][j];
      s += __shfl_xor(s, 8, 64);
      s += __shfl_xor(s, 16, 64);
      s += __shfl_xor(s, 32, 64);
      if (lane < 8) red[wave][k][sub * 8 + j] = s;
    }
    float sb = wave_sum(accb[k]);
    if (lane == 0) red[wave][k][64] = sb;
  }
  if constexpr (BN) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float s1 = sg[j], s2 = sgx[j];
      s1 += __shfl_xor(s1, 8, 64); s2 += __shfl_xor(s2, 8, 64);
      s1 += __shfl_xor(s1, 16, 64); s2 += __shfl_xor(s2, 16, 64);
      s1 += __shfl_xor(s1, 32, 64); s2 += __shfl_xor(s2, 32, 64);
      if (lane < 8) { bred[wave][sub * 8 + j][0] = s1; bred[wave][sub * 8 + j][1] = s2; }
    }
  }
  __syncthreads();
  // this block's partial row [NC][65] (dw row k, then db[k]); rows_sum_kernel adds the rows
  // in block order
  for (int idx = threadIdx.x; idx < NC * 65; idx += TPB) {
    const int k = idx / 65, c = idx % 65;
    float s = 0.f;
    for (int wv = 0; wv < TPB / 64; ++wv) s += red[wv][k][c];
    part[(long)blockIdx.x * NC * 65 + idx] = s;
  }
  if constexpr (BN) {
    if (threadIdx.x < 128) {
      const int c = threadIdx.x >> 1, q = threadIdx.x & 1;
      float s = 0.f;
      for (int wv = 0; wv < TPB / 64; ++wv) s += bred[wv][c][q];
      bn.part[((long)blockIdx.x * 64 + c) * 2 + q] = s;
    }
  }
}

// BN-backward apply of the decoder's last BatchNorm + ReLU from the head's gradient, which is
// recomputed per voxel from dlogits (da[v, c] = sum_k dl[k, v] w[k, c], rounded to T exactly as
// head_bwd_kernel would have stored it) instead of being written and read back:
// dy = k1 g + k2 xhat + k3, g = da [y sc + sh > 0] (bn_relu_bwd_apply_kernel's arithmetic).
template <typename T, bool NT, int NC>
__global__ void __launch_bounds__(TPB, 2) head_bn_apply_kernel(const T* y, const float* dlogits, const float* w,
                                                            const float* scale, const float* shift,
                                                            const float* mean, const float* invstd,
                                                            const float* coef, T* dy, long nvox_per_n, int N) {
  const long total = (long)N * nvox_per_n;
  const int sub = threadIdx.x & 7;
  // dy = k1 g + A (y - mean) + k3 with A = k2 invstd: the centred form (A y + (k3 - A mean)
  // loses ~eps |mean| / std to cancellation when |mean| >> std); six per-channel values held
  float sc[8], sh[8], k1[8], A[8], mu[8], k3[8], wk[NC][8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = sub * 8 + j;
    sc[j] = scale[c]; sh[j] = shift[c];
    k1[j] = coef[c * 3];
    A[j] = coef[c * 3 + 1] * invstd[c];
    mu[j] = mean[c];
    k3[j] = coef[c * 3 + 2];
#pragma unroll
    for (int k = 0; k < NC; ++k) wk[k][j] = w[k * 64 + c];
  }
  auto ld_dl = [&](const VoxQR& p, float (&dl)[NC]) {
#pragma unroll
    for (int k = 0; k < NC; ++k) dl[k] = dlogits[((long)p.q * NC + k) * nvox_per_n + p.r];
  };
  auto one = [&](long v, const float (&x)[8], const float (&dl)[NC]) {
    float o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = 0.f;
#pragma unroll
    for (int k = 0; k < NC; ++k)
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] += dl[k] * wk[k][j];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float g = (x[j] * sc[j] + sh[j] > 0.f) ? round_st<T>(o[j]) : 0.f;
      o[j] = k1[j] * g + (A[j] * (x[j] - mu[j]) + k3[j]);
    }
    head_st<T, NT>(dy + v * 64 + sub * 8, o);
  };
  const long stride = ((long)gridDim.x * blockDim.x) >> 3;
  long v = (blockIdx.x * (long)blockDim.x + threadIdx.x) >> 3;
  VoxQR pv(v, nvox_per_n);
#ifndef HEADA_U
#define HEADA_U 2
#endif
  constexpr int U = NC > 1 ? 1 : HEADA_U;  // (registers: 5 x 8 per-channel values + NC x 8 weights held)
#pragma unroll 1
  for (; v + (U - 1) * stride < total; v += U * stride) {
    float x[U][8], dl[U][NC];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      head_ld<T, NT>(y + (v + u * stride) * 64 + sub * 8, x[u]);
      ld_dl(u ? pv.plus((uint32_t)(u * stride)) : pv, dl[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) one(v + u * stride, x[u], dl[u]);
    pv.advance((uint32_t)(U * stride));
  }
  for (; v < total; v += stride) {
    float x[8], dl[NC];
    head_ld<T, NT>(y + v * 64 + sub * 8, x);
    ld_dl(pv, dl);
    one(v, x, dl);
    pv.advance((uint32_t)stride);
  }
}

// dw[k][c] += col (k, c), db[k] += col (k, 64) of the summed head partial rows
__global__ void head_bwd_finish_kernel(const float* sums, int ncls, float* dw, float* db) {
  const int idx = threadIdx.x;
  if (idx >= ncls * 65) return;
  const int k = idx / 65, c = idx % 65;
  if (c < 64) dw[k * 64 + c] += sums[idx];
  else db[k] += sums[idx];
}

// ---------------- losses ----------------
// partial rows: [block][4] = (sum p*t, sum p, sum t, sum bce)
__global__ void __launch_bounds__(TPB) loss_partial_kernel(const float* x, const float* t, long M, float* part) {
  __shared__ float red[4][TPB / 64];
  float a = 0.f, b = 0.f, c = 0.f, d = 0.f;
  auto one = [&](float xv, float tv) {
    const float p = 1.f / (1.f + expf(-xv));
    a += p * tv; b += p; c += tv;
    d += fmaxf(xv, 0.f) - xv * tv + log1pf(expf(-fabsf(xv)));
  };
  // 8 elements' loads in flight per trip, accumulated in the same element order as one at a
  // time (identical sums; one element per trip was a chain of 8 memory latencies per thread)
  const long stride = (long)gridDim.x * blockDim.x;
  long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  for (; i + 7 * stride < M; i += 8 * stride) {
    float xv[8], tv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) { xv[u] = x[i + u * stride]; tv[u] = t[i + u * stride]; }
#pragma unroll
    for (int u = 0; u < 8; ++u) one(xv[u], tv[u]);
  }
  for (; i < M; i += stride) one(x[i], t[i]);
  a = wave_sum(a); b = wave_sum(b); c = wave_sum(c); d = wave_sum(d);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) { red[0][wave] = a; red[1][wave] = b; red[2][wave] = c; red[3][wave] = d; }
  __syncthreads();
  if (threadIdx.x < 4) {
    float s = 0.f;
    for (int w = 0; w < TPB / 64; ++w) s += red[threadIdx.x][w];
    part[blockIdx.x * 4 + threadIdx.x] = s;
  }
}

// sums[0..3] (double) from partials; loss = wb*bce/M + wd*(1 - dice)
__global__ void loss_finalize_kernel(const float* part, int rows, long M, float smooth, float wb, float wd,
                                     double* sums, float* loss) {
  __shared__ double red[4][64];
  const int t = threadIdx.x;  // 256 threads: 4 sums x 64 lanes
  const int k = t >> 6, l = t & 63;
  double s = 0.0;
  for (int r = l; r < rows; r += 64) s += (double)part[r * 4 + k];
  red[k][l] = s;
  __syncthreads();
  if (t < 4) {
    double acc = 0.0;
    for (int i = 0; i < 64; ++i) acc += red[t][i];
    sums[t] = acc;
  }
  __syncthreads();
  if (t == 0) {
    const double I = sums[0], P = sums[1], Tt = sums[2], B = sums[3];
    const double dice = (2.0 * I + smooth) / (P + Tt + smooth);
    loss[0] = (float)(wb * (B / (double)M) + wd * (1.0 - dice));
  }
}

// dL/dx_i = gout * (wb*(p - t)/M + wd * -(2 t (P+T+s) - (2I+s)) / (P+T+s)^2 * p(1-p))
__global__ void loss_bwd_kernel(const float* x, const float* t, long M, const double* sums, float smooth,
                                float wb, float wd, const float* gout, float* dx) {
  const double I = sums[0], P = sums[1], Tt = sums[2];
  const double den = P + Tt + smooth, num = 2.0 * I + smooth;
  const float inv_den2 = (float)(1.0 / (den * den));
  const float fden = (float)den, fnum = (float)num;
  const float g = gout ? gout[0] : 1.f;
  const float invM = (float)(1.0 / (double)M);
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < M; i += (long)gridDim.x * blockDim.x) {
    const float xv = x[i], tv = t[i];
    const float p = 1.f / (1.f + expf(-xv));
    const float ddice_dp = -(2.f * tv * fden - fnum) * inv_den2;
    dx[i] = g * (wb * (p - tv) * invM + wd * ddice_dp * p * (1.f - p));
  }
}

// ---------------- Adam (torch.optim.Adam, foreach, coupled weight decay) ----------
// g_eff = g * s, s = gscale * (*gmul if gmul) (the data-parallel 1/world mean, the gradient-
// clip coefficient, the AMP unscale); when s != 1 the scaled gradient is also written back,
// so param.grad afterwards holds what torch's clip_grad_norm_ / DDP mean would leave there.
__global__ void adam_kernel(float* p, float* g, float* m, float* v, long n, AdamCoef c, const float* gmul) {
  const float s = gmul ? c.gscale * gmul[0] : c.gscale;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    float pi = p[i], gi = g[i], mi = m[i], vi = v[i];
    adam_update(pi, gi, mi, vi, c, s);
    if (s != 1.f) g[i] = gi;
    m[i] = mi;
    v[i] = vi;
    p[i] = pi;
  }
}

// The same over a list of [begin, end) element ranges of the flat buffers (the parameters the
// fused Adam + weight-pack kernels do not cover): blockIdx.y = range.
// p[b, e) = v for every [b, e) row of ranges (int64 pairs); grid.y = range
__global__ void fill_ranges_kernel(float* p, const long long* ranges, float v) {
  const long b = ranges[2 * blockIdx.y], e = ranges[2 * blockIdx.y + 1];
  for (long i = b + blockIdx.x * (long)blockDim.x + threadIdx.x; i < e; i += (long)gridDim.x * blockDim.x) p[i] = v;
}

__global__ void adam_ranges_kernel(float* p, float* g, float* m, float* v, const long long* ranges, AdamCoef c,
                                   const float* gmul) {
  const float s = gmul ? c.gscale * gmul[0] : c.gscale;
  const long b = ranges[2 * blockIdx.y], e = ranges[2 * blockIdx.y + 1];
  for (long i = b + blockIdx.x * (long)blockDim.x + threadIdx.x; i < e; i += (long)gridDim.x * blockDim.x) {
    float pi = p[i], gi = g[i], mi = m[i], vi = v[i];
    adam_update(pi, gi, mi, vi, c, s);
    if (s != 1.f) g[i] = gi;
    m[i] = mi;
    v[i] = vi;
    p[i] = pi;
  }
}

// ---------------- global gradient norm / clip (torch.nn.utils.clip_grad_norm_) ----------
// pass 1: per-block fp64 partial sums of g^2 (fp32 squares), one row per block
constexpr int kNormBlocks = 1024;
__global__ void __launch_bounds__(TPB) sumsq_kernel(const float* g, long n, double* part) {
  __shared__ double red[TPB / 64];
  double s = 0.0;
  const long n4 = n / 4;
  const f32x4_t* g4 = reinterpret_cast<const f32x4_t*>(g);
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    const f32x4_t v = g4[i];
    s += (double)(v[0] * v[0]) + (double)(v[1] * v[1]) + (double)(v[2] * v[2]) + (double)(v[3] * v[3]);
  }
  if (blockIdx.x == 0)
    for (long i = n4 * 4 + threadIdx.x; i < n; i += blockDim.x) s += (double)(g[i] * g[i]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int w = 0; w < TPB / 64; ++w) t += red[w];
    part[blockIdx.x] = t;
  }
}
// pass 2 (one block): norm = gscale * sqrt(sum of rows, in row order); mul = gscale *
// min(1, max_norm / (norm + 1e-6)) (clip_grad_norm_'s clamped coefficient; max_norm <= 0:
// no clipping, mul = gscale)
__global__ void clip_finalize_kernel(const double* part, int rows, float gscale, float max_norm, float* norm_out,
                                     float* mul_out) {
  __shared__ double red[256];
  double s = 0.0;
  for (int r = threadIdx.x; r < rows; r += 256) s += part[r];
  red[threadIdx.x] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int i = 0; i < 256; ++i) t += red[i];
    const float norm = (float)sqrt(t) * gscale;
    float coef = 1.f;
    if (max_norm > 0.f) coef = fminf(1.f, max_norm / (norm + 1e-6f));
    if (norm_out) norm_out[0] = norm;
    if (mul_out) mul_out[0] = gscale * coef;
  }
}
// g *= *mul (in place)
__global__ void scale_kernel(float* g, long n, const float* mul) {
  const float s = mul[0];
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) g[i] *= s;
}

// fp32 split-K slabs [splits][nvox][C] -> sum in split order + bias, store T, BN partial
// sums; 64 voxels per block row
constexpr int kMaxSplitSlabs = 16;  // slabs loaded together (more: summed one by one after)
// 16 voxel lanes x 64 channels per block: a thread owns 4 of the row's 64 voxels, so a voxel
// row is 4 rounds of slab loads instead of 16 (deep levels have few rows: level 4 is 8 rows x
// 16 channel blocks, and each round is a full memory latency)
constexpr int kSeThreads = 1024;
#ifndef SE_BATCH
#define SE_BATCH 0
#endif
template <typename T>
__global__ void __launch_bounds__(kSeThreads) split_epilogue_kernel(const float* acc, int splits, const float* bias,
                                                                    T* y0, T* y1, int cy0, float* stats, int C,
                                                                    long nvox, int relu) {
  // stats row = (sum, M2 about the row mean), count row after the [rows][C][2] block
  constexpr int NV = kSeThreads / 64, KPT = 64 / NV;
  __shared__ float red[NV][64][3];
  const int cl = threadIdx.x & 63, vl = threadIdx.x >> 6;
  const int c = blockIdx.y * 64 + cl;
  const long v0 = (long)blockIdx.x * 64;
  const float bc = bias ? bias[c] : 0.f;
  float xs[KPT];
  float s1 = 0.f, s2 = 0.f;
  int cntv = 0;
#if SE_BATCH
  // every slab load of the thread's KPT voxels issued before the first add: the store of a
  // voxel may alias the next voxel's slabs for the compiler, so the per-voxel loop below ran
  // KPT rounds of memory latency (same summation order either way)
  float part[KPT][kMaxSplitSlabs];
#pragma unroll
  for (int i = 0; i < KPT; ++i) {
    const long v = v0 + vl + i * NV;
#pragma unroll
    for (int sp = 0; sp < kMaxSplitSlabs; ++sp)
      if (sp < splits && v < nvox) part[i][sp] = acc[((long)sp * nvox + v) * C + c];
  }
#endif
#pragma unroll
  for (int i = 0; i < KPT; ++i) {
    const long v = v0 + vl + i * NV;
    xs[i] = 0.f;
    if (v >= nvox) continue;
#if SE_BATCH
    float x = part[i][0];
#pragma unroll
    for (int sp = 1; sp < kMaxSplitSlabs; ++sp)
      if (sp < splits) x += part[i][sp];
#else
    // the split slabs in split order (a fixed summation order); all of a voxel's slab loads
    // are issued before the first add (a load -> add chain per slab was latency-bound)
    float part[kMaxSplitSlabs];
#pragma unroll
    for (int sp = 0; sp < kMaxSplitSlabs; ++sp)
      if (sp < splits) part[sp] = acc[((long)sp * nvox + v) * C + c];
    float x = part[0];
#pragma unroll
    for (int sp = 1; sp < kMaxSplitSlabs; ++sp)
      if (sp < splits) x += part[sp];
#endif
    for (int sp = kMaxSplitSlabs; sp < splits; ++sp) x += acc[((long)sp * nvox + v) * C + c];
    x += bc;
    if (relu) x = fmaxf(x, 0.f);
    T* dst = c < cy0 ? y0 + v * cy0 + c : y1 + v * (C - cy0) + (c - cy0);
    Elem<T>::st(dst, x);
    xs[i] = x;
    s1 += x;
    ++cntv;
  }
  if (!stats) return;
  const float m = cntv ? s1 / cntv : 0.f;
  float sd = 0.f;
#pragma unroll
  for (int i = 0; i < KPT; ++i)
    if (v0 + vl + i * NV < nvox) { s2 += (xs[i] - m) * (xs[i] - m); sd += xs[i] - m; }
  if (cntv) s2 -= sd * sd / cntv;  // deviations about the rounded mean
  red[vl][cl][0] = s1;
  red[vl][cl][1] = s2;
  red[vl][cl][2] = (float)cntv;
  __syncthreads();
  if (vl == 0) {
    float S = 0.f, Nn = 0.f;
    for (int k = 0; k < NV; ++k) { S += red[k][cl][0]; Nn += red[k][cl][2]; }
    const float mb = Nn > 0.f ? S / Nn : 0.f;
    float M2 = 0.f, sdd = 0.f;
    for (int k = 0; k < NV; ++k) {
      const float n = red[k][cl][2];
      if (n > 0.f) {
        const float d = red[k][cl][0] / n - mb;
        M2 += red[k][cl][1] + n * d * d;
        sdd += n * d;
      }
    }
    if (Nn > 0.f) M2 -= sdd * sdd / Nn;
    stats[((long)blockIdx.x * C + c) * 2] = S;
    stats[((long)blockIdx.x * C + c) * 2 + 1] = M2;
    if (cl == 0 && blockIdx.y == 0) stats[(long)gridDim.x * C * 2 + blockIdx.x] = Nn;
  }
}

// ---------------- NDHWC (T, Cs stored channels) -> NCDHW fp32, first C channels ----------
template <typename T>
__global__ void unpack_output_kernel(const T* in, float* out, int N, int C, int Cs, long V) {
  const long total = (long)N * C * V;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long v = i % V, nc = i / V;
    const int c = (int)(nc % C);
    const long n = nc / C;
    out[i] = Elem<T>::ld(in + (n * V + v) * Cs + c);
  }
}

template <typename T>
__global__ void add_kernel(T* dst, const T* src, long nvec) {
  constexpr int VEC = Elem<T>::kVec;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < nvec; i += (long)gridDim.x * blockDim.x) {
    float a[VEC], b[VEC];
    load16<T>(dst + i * VEC, a);
    load16<T>(src + i * VEC, b);
#pragma unroll
    for (int j = 0; j < VEC; ++j) a[j] += b[j];
    store16<T>(dst + i * VEC, a);
  }
}

// the head kernels with n_classes as a template argument (1..4)
template <int NC, typename F>
int with_ncls(int ncls, F&& f) {
  if constexpr (NC > 4) {
    return -1;
  } else {
    if (ncls == NC) { f(std::integral_constant<int, NC>{}); return 0; }
    return with_ncls<NC + 1>(ncls, f);
  }
}
template <typename T, bool BN>
int launch_head_fwd(bool nt, int grid, hipStream_t s, const void* a, const float* w, const float* b, float* out,
                    long nvox_per_n, int N, int ncls, int act, float thr, const float* sc, const float* sh) {
  return with_ncls<1>(ncls, [&](auto nc) {
    constexpr int NC = decltype(nc)::value;
    hipLaunchKernelGGL((nt ? head_fwd_kernel<T, true, BN, NC> : head_fwd_kernel<T, false, BN, NC>), dim3(grid),
                       dim3(TPB), 0, s, (const T*)a, w, b, out, nvox_per_n, N, act, thr, sc, sh);
  });
}
template <typename T, bool BN>
int launch_head_bwd(bool nt, int grid, hipStream_t s, const void* a, const float* dl, const float* w, void* da,
                    float* part, long nvox_per_n, int N, int ncls, const HeadBN& bn) {
  return with_ncls<1>(ncls, [&](auto nc) {
    constexpr int NC = decltype(nc)::value;
    hipLaunchKernelGGL((nt ? head_bwd_kernel<T, true, BN, NC> : head_bwd_kernel<T, false, BN, NC>), dim3(grid),
                       dim3(TPB), 0, s, (const T*)a, dl, w, (T*)da, part, nvox_per_n, N, bn);
  });
}
template <typename T>
int launch_head_apply(bool nt, int grid, hipStream_t s, const void* y, const float* dl, const float* w,
                      const float* sc, const float* sh, const float* mu, const float* is, const float* coef, void* dy,
                      long nvox_per_n, int N, int ncls) {
  return with_ncls<1>(ncls, [&](auto nc) {
    constexpr int NC = decltype(nc)::value;
    hipLaunchKernelGGL((nt ? head_bn_apply_kernel<T, true, NC> : head_bn_apply_kernel<T, false, NC>), dim3(grid),
                       dim3(TPB), 0, s, (const T*)y, dl, w, sc, sh, mu, is, coef, (T*)dy, nvox_per_n, N);
  });
}

}  // namespace

extern "C" {

int pcms_pack_input(int dtype, const float* in, void* out, int N, int Cin, long V, int Cp, hipStream_t s) {
  if (Cp == 8 && Cin <= 8 && V % 4 == 0 && ((uintptr_t)in & 15) == 0 && ((uintptr_t)out & 15) == 0) {
    const int grid = grid_for((long)N * V / 4, TPB, 16 * 256);  // ~one quad per thread: every load in flight at once
    if (dtype == PCMS_BF16) hipLaunchKernelGGL(pack_input4_kernel<bf16_t>, dim3(grid), dim3(TPB), 0, s, in, (bf16_t*)out, N, Cin, V);
    else hipLaunchKernelGGL(pack_input4_kernel<float>, dim3(grid), dim3(TPB), 0, s, in, (float*)out, N, Cin, V);
    PCMS_CHECK_LAUNCH();
  }
  const int grid = grid_for((long)N * V, TPB);
  if (dtype == PCMS_BF16) hipLaunchKernelGGL(pack_input_kernel<bf16_t>, dim3(grid), dim3(TPB), 0, s, in, (bf16_t*)out, N, Cin, V, Cp);
  else hipLaunchKernelGGL(pack_input_kernel<float>, dim3(grid), dim3(TPB), 0, s, in, (float*)out, N, Cin, V, Cp);
  PCMS_CHECK_LAUNCH();
}

int pcms_bn_finalize(const float* part, int rows, int C, double count, const float* gamma, const float* beta,
                     float* rmean, float* rvar, long long* nbt, float momentum, float eps,
                     float* scale, float* shift, float* mean, float* invstd, double* ws, hipStream_t s) {
  if (rows <= kSmallRows) {
    hipLaunchKernelGGL(colsum_finalize_small_kernel<false>, dim3(cdiv(C, 64)), dim3(64 * kCfRL), 0, s, part, rows, C,
                       part + (long)rows * C * 2, count, gamma, beta, rmean, rvar, nbt, momentum, eps, scale, shift,
                       mean, invstd, nullptr, nullptr, nullptr);
    PCMS_CHECK_LAUNCH();
  }
  hipLaunchKernelGGL(colsum2_kernel, dim3(cdiv(C, 64), kRB), dim3(256), 0, s, part, rows, C,
                     part + (long)rows * C * 2, ws);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(bn_finalize_kernel, dim3(cdiv(C, 64)), dim3(64), 0, s, (const double*)ws, C, count, gamma,
                     beta, rmean, rvar, nbt, momentum, eps, scale, shift, mean, invstd);
  PCMS_CHECK_LAUNCH();
}

int pcms_bn_ws_doubles(int C) { return kRB * C * 2; }

int pcms_bn_fold(const float* w, const float* b, const float* gamma, const float* beta, const float* rmean,
                 const float* rvar, float eps, int Cout, long K, float* wo, float* bo, hipStream_t s) {
  if (Cout <= 0 || K <= 0) return -1;
  hipLaunchKernelGGL(bn_fold_kernel, dim3(grid_for(K, 256, 64), Cout), dim3(256), 0, s, w, b, gamma, beta, rmean, rvar,
                     eps, Cout, K, wo, bo);
  PCMS_CHECK_LAUNCH();
}

int pcms_bn_eval_coeffs(const float* gamma, const float* beta, const float* rmean, const float* rvar, float eps,
                        int C, float* scale, float* shift, hipStream_t s) {
  hipLaunchKernelGGL(bn_eval_coeffs_kernel, dim3(cdiv(C, 256)), dim3(256), 0, s, gamma, beta, rmean, rvar, eps, C, scale, shift);
  PCMS_CHECK_LAUNCH();
}

static int ew_grid(int dtype, int C, long nvox) {
  const int VEC = dtype == PCMS_BF16 ? 8 : 4;
  const int VL = TPB / (C / VEC);
  return grid_for(nvox, VL * 4, 8192);
}

int pcms_bn_relu(int dtype, const void* y, void* a, const float* scale, const float* shift, int C, long nvox,
                 hipStream_t s) {
  const int VEC = dtype == PCMS_BF16 ? 8 : 4;
  if (C % VEC || TPB % (C / VEC)) return -1;
  const int grid = ew_grid(dtype, C, nvox);
  const bool nt = nvox * C * (dtype == PCMS_BF16 ? 2 : 4) >= kNtBytesBn;
  if (dtype == PCMS_BF16)
    hipLaunchKernelGGL((nt ? bn_relu_kernel<bf16_t, true> : bn_relu_kernel<bf16_t, false>), dim3(grid), dim3(TPB), 0, s,
                       (const bf16_t*)y, (bf16_t*)a, scale, shift, C, nvox);
  else
    hipLaunchKernelGGL((nt ? bn_relu_kernel<float, true> : bn_relu_kernel<float, false>), dim3(grid), dim3(TPB), 0, s,
                       (const float*)y, (float*)a, scale, shift, C, nvox);
  PCMS_CHECK_LAUNCH();
}

// the BN-backward reduce passes' block cap (their partial-row count): kSmallRows (512, the
// product: the finalize is one launch; round 6 kernel trace -15 us per step vs 2048,
// profiles/r6_bn_rows_cap_ab.txt) or more (two-stage finalize); A/B switch: v <= 0 queries,
// returns the old value; set before the workspace queries
#ifndef PCMS_BN_ROWS_CAP
#define PCMS_BN_ROWS_CAP 512
#endif
static int g_bn_rows_cap = PCMS_BN_ROWS_CAP;
int pcms_bn_bwd_rows_cap(int v) {
  const int old = g_bn_rows_cap;
  if (v > 0) g_bn_rows_cap = v;
  return old;
}

// number of partial rows pcms_bn_relu_bwd_reduce writes (caller sizes `part`)
int pcms_bn_bwd_rows(int dtype, int C, long nvox) {
  const int VEC = dtype == PCMS_BF16 ? 8 : 4;
  const int VL = TPB / (C / VEC);
  // small (deep) grids: one trip of 4 rows per thread and 4x the blocks (a block's reduction
  // is a chain of memory latencies), as long as the rows stay on the one-launch finalize
  const int small = grid_for(nvox, VL * 4, 2048);
  return small <= kSmallRows ? small : grid_for(nvox, VL * 16, g_bn_rows_cap);
}

int pcms_bn_relu_bwd(int dtype, const void* da, const void* y, const float* scale, const float* shift,
                     const float* mean, const float* invstd, const float* gamma, float* part, float* coef,
                     float* dgamma, float* dbeta, void* dy, int C, long nvox, double* ws, hipStream_t s) {
  const int VEC = dtype == PCMS_BF16 ? 8 : 4;
  if (C % VEC || (TPB % (C / VEC)) != 0) return -1;
  const int rows = pcms_bn_bwd_rows(dtype, C, nvox);
  // the reduce keeps the default cache policy: what it leaves in the Infinity Cache the apply
  // pass below re-reads (measured: nt here 99 us but the apply 118 -> 135 us at level 0)
  if (dtype == PCMS_BF16)
    hipLaunchKernelGGL((bn_relu_bwd_reduce_kernel<bf16_t, false>), dim3(rows), dim3(TPB), 0, s, (const bf16_t*)da, (const bf16_t*)y, scale, shift, mean, invstd, part, C, nvox);
  else
    hipLaunchKernelGGL((bn_relu_bwd_reduce_kernel<float, false>), dim3(rows), dim3(TPB), 0, s, (const float*)da, (const float*)y, scale, shift, mean, invstd, part, C, nvox);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  return pcms_bn_relu_bwd_finish(dtype, da, y, scale, shift, mean, invstd, gamma, part, rows, coef, dgamma, dbeta,
                                 dy, C, nvox, ws, s);
}

int pcms_bn_relu_bwd_finish(int dtype, const void* da, const void* y, const float* scale, const float* shift,
                            const float* mean, const float* invstd, const float* gamma, const float* part, int rows,
                            float* coef, float* dgamma, float* dbeta, void* dy, int C, long nvox, double* ws,
                            hipStream_t s) {
  const int VEC = dtype == PCMS_BF16 ? 8 : 4;
  if (C % VEC || (TPB % (C / VEC)) != 0) return -1;
  const bool nt = nvox * C * (dtype == PCMS_BF16 ? 2 : 4) >= kNtBytesBn;
  hipError_t e;
  if (rows <= kSmallRows) {
    hipLaunchKernelGGL(colsum_finalize_small_kernel<true>, dim3(cdiv(C, 64)), dim3(64 * kCfRL), 0, s, part, rows, C,
                       (const float*)nullptr, (double)nvox, gamma, nullptr, nullptr, nullptr, nullptr, 0.f, 0.f,
                       nullptr, nullptr, nullptr, const_cast<float*>(invstd), dgamma, dbeta, coef);
  } else {
    hipLaunchKernelGGL(colsum2_kernel, dim3(cdiv(C, 64), kRB), dim3(256), 0, s, (const float*)part, rows, C,
                       (const float*)nullptr, ws);
    e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
    hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3(cdiv(C, 64)), dim3(64), 0, s, (const double*)ws, C,
                       (double)nvox, gamma, invstd, dgamma, dbeta, coef);
  }
  e = hipGetLastError();
  if (e != hipSuccess || dy == nullptr) return (int)e;  // dy NULL: the consumer applies (coef)
  const int grid = ew_grid(dtype, C, nvox);
  if (dtype == PCMS_BF16)
    hipLaunchKernelGGL((nt ? bn_relu_bwd_apply_kernel<bf16_t, true> : bn_relu_bwd_apply_kernel<bf16_t, false>), dim3(grid), dim3(TPB), 0, s, (const bf16_t*)da, (const bf16_t*)y, scale, shift, mean, invstd, (const float*)coef, (bf16_t*)dy, C, nvox);
  else
    hipLaunchKernelGGL((nt ? bn_relu_bwd_apply_kernel<float, true> : bn_relu_bwd_apply_kernel<float, false>), dim3(grid), dim3(TPB), 0, s, (const float*)da, (const float*)y, scale, shift, mean, invstd, (const float*)coef, (float*)dy, C, nvox);
  PCMS_CHECK_LAUNCH();
}

// grid of the cell kernels: a multiple of CV / gcd so every thread keeps one channel group
static int cell_grid(long total, int CV, int cap) {
  int g = grid_for(total, TPB, cap);
  const int per = CV / std::__gcd(CV, TPB);  // blocks per period of cv
  return std::max(per, g / per * per);
}

int pcms_bn_relu_pool(int dtype, const void* y, void* a, void* p, const float* scale, const float* shift, int N,
                      int D, int H, int W, int C, hipStream_t s) {
  const int VEC = dtype == PCMS_BF16 ? 8 : 4;
  if (C % VEC) return -1;
  const long cells = (long)N * ((D + 1) / 2) * ((H + 1) / 2) * ((W + 1) / 2);
  if (cells * 8 >= (1L << 31)) return -7;  // 32-bit index math in the kernel
  const int CV = C / VEC;
  const int grid = cell_grid(cells * CV, CV, 8192);
  const bool nt = (long)N * D * H * W * C * (dtype == PCMS_BF16 ? 2 : 4) >= kNtBytesBn;
  if (dtype == PCMS_BF16)
    hipLaunchKernelGGL((nt ? bn_relu_pool_kernel<bf16_t, true> : bn_relu_pool_kernel<bf16_t, false>), dim3(grid),
                       dim3(TPB), 0, s, (const bf16_t*)y, (bf16_t*)a, (bf16_t*)p, scale, shift, N, D, H, W, C);
  else
    hipLaunchKernelGGL((nt ? bn_relu_pool_kernel<float, true> : bn_relu_pool_kernel<float, false>), dim3(grid),
                       dim3(TPB), 0, s, (const float*)y, (float*)a, (float*)p, scale, shift, N, D, H, W, C);
  PCMS_CHECK_LAUNCH();
}

int pcms_maxpool_bwd_bn_rows(int dtype, int N, int D, int H, int W, int C) {
  const int VEC = dtype == PCMS_BF16 ? 8 : 4;
  const long cells = (long)N * ((D + 1) / 2) * ((H + 1) / 2) * ((W + 1) / 2);
  return cell_grid(cells * (C / VEC), C / VEC, g_bn_rows_cap);
}

int pcms_maxpool_bwd_bn(int dtype, const void* y, const float* scale, const float* shift, const float* mean,
                        const float* invstd, const void* dp, void* da, float* part, int N, int D, int H, int W,
                        int C, hipStream_t s) {
  const int VEC = dtype == PCMS_BF16 ? 8 : 4;
  if (C % VEC || TPB % (C / VEC)) return -1;
  const long cells = (long)N * ((D + 1) / 2) * ((H + 1) / 2) * ((W + 1) / 2);
  if (cells * 8 >= (1L << 31)) return -7;
  const int grid = pcms_maxpool_bwd_bn_rows(dtype, N, D, H, W, C);
  if (dtype == PCMS_BF16)
    hipLaunchKernelGGL(maxpool_bwd_bn_kernel<bf16_t>, dim3(grid), dim3(TPB), 0, s, (const bf16_t*)y, scale, shift,
                       mean, invstd, (const bf16_t*)dp, (bf16_t*)da, part, N, D, H, W, C);
  else
    hipLaunchKernelGGL(maxpool_bwd_bn_kernel<float>, dim3(grid), dim3(TPB), 0, s, (const float*)y, scale, shift,
                       mean, invstd, (const float*)dp, (float*)da, part, N, D, H, W, C);
  PCMS_CHECK_LAUNCH();
}

int pcms_maxpool_bwd_bn_sums(int dtype, const void* y, const float* scale, const float* shift, const float* mean,
                             const float* invstd, const void* dp, const void* da, float* part, int N, int D, int H,
                             int W, int C, hipStream_t s) {
  const int VEC = dtype == PCMS_BF16 ? 8 : 4;
  if (C % VEC || TPB % (C / VEC)) return -1;
  const long cells = (long)N * ((D + 1) / 2) * ((H + 1) / 2) * ((W + 1) / 2);
  if (cells * 8 >= (1L << 31)) return -7;
  const int grid = pcms_maxpool_bwd_bn_rows(dtype, N, D, H, W, C);
  if (dtype == PCMS_BF16)
    hipLaunchKernelGGL((maxpool_bwd_bn_kernel<bf16_t, false>), dim3(grid), dim3(TPB), 0, s, (const bf16_t*)y, scale,
                       shift, mean, invstd, (const bf16_t*)dp, (bf16_t*)const_cast<void*>(da), part, N, D, H, W, C);
  else
    hipLaunchKernelGGL((maxpool_bwd_bn_kernel<float, false>), dim3(grid), dim3(TPB), 0, s, (const float*)y, scale,
                       shift, mean, invstd, (const float*)dp, (float*)const_cast<void*>(da), part, N, D, H, W, C);
  PCMS_CHECK_LAUNCH();
}

int pcms_maxpool_bn_apply(int dtype, const void* y, const float* scale, const float* shift, const float* mean,
                          const float* invstd, const float* coef, const void* dp, const void* da, void* dy, int N,
                          int D, int H, int W, int C, hipStream_t s) {
  const int VEC = dtype == PCMS_BF16 ? 8 : 4;
  if (C % VEC || TPB % (C / VEC)) return -1;
  const long cells = (long)N * ((D + 1) / 2) * ((H + 1) / 2) * ((W + 1) / 2);
  if (cells * 8 >= (1L << 31)) return -7;
  const int CV = C / VEC;
  const int grid = cell_grid(cells * CV, CV, 8192);
  const bool nt = (long)N * D * H * W * C * (dtype == PCMS_BF16 ? 2 : 4) >= kNtBytesBn;
  if (dtype == PCMS_BF16)
    hipLaunchKernelGGL((nt ? maxpool_bn_apply_kernel<bf16_t, true> : maxpool_bn_apply_kernel<bf16_t, false>),
                       dim3(grid), dim3(TPB), 0, s, (const bf16_t*)y, scale, shift, mean, invstd, coef,
                       (const bf16_t*)dp, (const bf16_t*)da, (bf16_t*)dy, N, D, H, W, C);
  else
    hipLaunchKernelGGL((nt ? maxpool_bn_apply_kernel<float, true> : maxpool_bn_apply_kernel<float, false>),
                       dim3(grid), dim3(TPB), 0, s, (const float*)y, scale, shift, mean, invstd, coef,
                       (const float*)dp, (const float*)da, (float*)dy, N, D, H, W, C);
  PCMS_CHECK_LAUNCH();
}

int pcms_maxpool_fwd(int dtype, const void* a, void* p, int N, int D, int H, int W, int C, hipStream_t s) {
  if ((long)N * D * H * W * C >= (1L << 31)) return -7;  // 32-bit index math in the kernel
  const int VEC = dtype == PCMS_BF16 ? 8 : 4;
  const long total = (long)N * (D / 2) * (H / 2) * (W / 2) * (C / VEC);
  const int grid = grid_for(total, TPB);
  if (dtype == PCMS_BF16) hipLaunchKernelGGL(maxpool_fwd_kernel<bf16_t>, dim3(grid), dim3(TPB), 0, s, (const bf16_t*)a, (bf16_t*)p, N, D, H, W, C);
  else hipLaunchKernelGGL(maxpool_fwd_kernel<float>, dim3(grid), dim3(TPB), 0, s, (const float*)a, (float*)p, N, D, H, W, C);
  PCMS_CHECK_LAUNCH();
}

int pcms_maxpool_bwd(int dtype, const void* a, const void* dp, void* da, int N, int D, int H, int W, int C,
                     hipStream_t s) {
  if ((long)N * D * H * W * C >= (1L << 31)) return -7;  // 32-bit index math in the kernel
  const int VEC = dtype == PCMS_BF16 ? 8 : 4;
  const long total = (long)N * (D / 2) * (H / 2) * (W / 2) * (C / VEC);
  const int grid = grid_for(total, TPB);
  if (dtype == PCMS_BF16) hipLaunchKernelGGL(maxpool_bwd_kernel<bf16_t>, dim3(grid), dim3(TPB), 0, s, (const bf16_t*)a, (const bf16_t*)dp, (bf16_t*)da, N, D, H, W, C);
  else hipLaunchKernelGGL(maxpool_bwd_kernel<float>, dim3(grid), dim3(TPB), 0, s, (const float*)a, (const float*)dp, (float*)da, N, D, H, W, C);
  PCMS_CHECK_LAUNCH();
}

static int box_sum_rows(int dtype, int N, int C, int bd, int bh, int bw) {
  const int VEC = dtype == PCMS_BF16 ? 8 : 4;
  const int VL = TPB / (C / VEC);
  return grid_for((long)N * bd * bh * bw, VL * 8, 1024);
}
int pcms_box_channel_sum_ws_floats(int dtype, int N, int C, int bd, int bh, int bw) {
  return box_sum_rows(dtype, N, C, bd, bh, bw) * C;
}

int pcms_box_channel_sum(int dtype, const void* x, float* out, float* ws, int N, int D, int H, int W, int C,
                         int z0, int y0, int x0, int bd, int bh, int bw, hipStream_t s) {
  if ((long)N * D * H * W >= (1L << 31)) return -7;  // 32-bit index math in the kernel
  const int VEC = dtype == PCMS_BF16 ? 8 : 4;
  if (C % VEC || TPB % (C / VEC)) return -1;
  if (ws == nullptr) return -2;
  const int grid = box_sum_rows(dtype, N, C, bd, bh, bw);
  if (dtype == PCMS_BF16) hipLaunchKernelGGL(box_channel_sum_kernel<bf16_t>, dim3(grid), dim3(TPB), 0, s, (const bf16_t*)x, ws, N, D, H, W, C, z0, y0, x0, bd, bh, bw);
  else hipLaunchKernelGGL(box_channel_sum_kernel<float>, dim3(grid), dim3(TPB), 0, s, (const float*)x, ws, N, D, H, W, C, z0, y0, x0, bd, bh, bw);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(rows_sum_kernel<true>, dim3(cdiv(C, 8)), dim3(256), 0, s, (const float*)ws, grid, C, out);
  PCMS_CHECK_LAUNCH();
}

static int head_fwd_any(int dtype, const void* a, const float* w, const float* b, float* out, long nvox_per_n,
                        int N, int ncls, int act, float thr, const float* sc, const float* sh, hipStream_t s) {
  if ((long)N * nvox_per_n >= (1L << 31)) return -7;  // 32-bit index math in the kernel
  if (act < 0 || act > 2) return -1;
  const int grid = grid_for((long)N * nvox_per_n * 8, TPB);
  const bool nt = (long)N * nvox_per_n * 64 * (dtype == PCMS_BF16 ? 2 : 4) >= kNtBytes;
  const bool bn = sc != nullptr;
  int rc;
  if (dtype == PCMS_BF16)
    rc = bn ? launch_head_fwd<bf16_t, true>(nt, grid, s, a, w, b, out, nvox_per_n, N, ncls, act, thr, sc, sh)
            : launch_head_fwd<bf16_t, false>(nt, grid, s, a, w, b, out, nvox_per_n, N, ncls, act, thr, sc, sh);
  else
    rc = bn ? launch_head_fwd<float, true>(nt, grid, s, a, w, b, out, nvox_per_n, N, ncls, act, thr, sc, sh)
            : launch_head_fwd<float, false>(nt, grid, s, a, w, b, out, nvox_per_n, N, ncls, act, thr, sc, sh);
  if (rc) return rc;
  PCMS_CHECK_LAUNCH();
}

int pcms_head_fwd(int dtype, const void* a, const float* w, const float* b, float* out, long nvox_per_n, int N,
                  int ncls, int act, float thr, hipStream_t s) {
  return head_fwd_any(dtype, a, w, b, out, nvox_per_n, N, ncls, act, thr, nullptr, nullptr, s);
}

int pcms_head_bn_fwd(int dtype, const void* y, const float* scale, const float* shift, const float* w,
                     const float* b, float* out, long nvox_per_n, int N, int ncls, int act, float thr,
                     hipStream_t s) {
  if (scale == nullptr || shift == nullptr) return -2;
  return head_fwd_any(dtype, y, w, b, out, nvox_per_n, N, ncls, act, thr, scale, shift, s);
}

static int head_bwd_rows(long nvox) { return grid_for(nvox * 8, TPB, 2048); }

// the head partial rows [grid][ncls][65] -> dw[k][c] += (k, c), db[k] += (k, 64)
static int head_finish(int grid, float* ws, int ncls, float* dw, float* db, hipStream_t s) {
  float* sums = ws + (long)grid * ncls * 65;
  hipLaunchKernelGGL(rows_sum_kernel<false>, dim3(cdiv(ncls * 65, 8)), dim3(256), 0, s, (const float*)ws, grid, ncls * 65,
                     sums);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(head_bwd_finish_kernel, dim3(1), dim3(320), 0, s, (const float*)sums, ncls, dw, db);
  PCMS_CHECK_LAUNCH();
}
// workspace: the per-block partial rows + one summed row
int pcms_head_bwd_ws_floats(long nvox_per_n, int N, int ncls) {
  return (head_bwd_rows((long)N * nvox_per_n) + 1) * ncls * 65;
}

int pcms_head_bwd(int dtype, const void* a, const float* dlogits, const float* w, void* da, float* dw, float* db,
                  float* ws, long nvox_per_n, int N, int ncls, hipStream_t s) {
  if ((long)N * nvox_per_n >= (1L << 31)) return -7;  // 32-bit index math in the kernel
  if (ncls > 4 || ncls < 1) return -1;
  if (ws == nullptr) return -2;
  const int grid = head_bwd_rows((long)N * nvox_per_n);
  const bool nt = (long)N * nvox_per_n * 64 * (dtype == PCMS_BF16 ? 2 : 4) >= kNtBytes;
  const HeadBN nobn{};
  if (dtype == PCMS_BF16) launch_head_bwd<bf16_t, false>(nt, grid, s, a, dlogits, w, da, ws, nvox_per_n, N, ncls, nobn);
  else launch_head_bwd<float, false>(nt, grid, s, a, dlogits, w, da, ws, nvox_per_n, N, ncls, nobn);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  return head_finish(grid, ws, ncls, dw, db, s);
}

int pcms_head_bn_bwd_rows(long nvox_per_n, int N) { return head_bwd_rows((long)N * nvox_per_n); }

int pcms_head_bn_bwd(int dtype, const void* y, const float* scale, const float* shift, const float* mean,
                     const float* invstd, const float* gamma, const float* dlogits, const float* w, float* dw,
                     float* db, float* ws, float* bnpart, float* coef, float* dgamma, float* dbeta, void* dy,
                     long nvox_per_n, int N, int ncls, double* bnws, hipStream_t s) {
  if ((long)N * nvox_per_n >= (1L << 31)) return -7;  // 32-bit index math in the kernels
  if (ncls > 4 || ncls < 1) return -1;
  if (ws == nullptr || bnpart == nullptr || bnws == nullptr || coef == nullptr) return -2;
  const long nvox = (long)N * nvox_per_n;
  const int grid = head_bwd_rows(nvox);
  const bool nt = nvox * 64 * (dtype == PCMS_BF16 ? 2 : 4) >= kNtBytes;
  const HeadBN bn{scale, shift, mean, invstd, bnpart};
  // pass 1: head weight / bias partials + BatchNorm-backward partial sums (reads y2, dlogits)
  if (dtype == PCMS_BF16) launch_head_bwd<bf16_t, true>(false, grid, s, y, dlogits, w, nullptr, ws, nvox_per_n, N, ncls, bn);
  else launch_head_bwd<float, true>(false, grid, s, y, dlogits, w, nullptr, ws, nvox_per_n, N, ncls, bn);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  if ((e = (hipError_t)head_finish(grid, ws, ncls, dw, db, s)) != hipSuccess) return (int)e;
  hipLaunchKernelGGL(colsum2_kernel, dim3(1, kRB), dim3(256), 0, s, (const float*)bnpart, grid, 64,
                     (const float*)nullptr, bnws);
  if ((e = hipGetLastError()) != hipSuccess) return (int)e;
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3(1), dim3(64), 0, s, (const double*)bnws, 64, (double)nvox, gamma,
                     invstd, dgamma, dbeta, coef);
  if ((e = hipGetLastError()) != hipSuccess) return (int)e;
  // pass 2: dy of the BatchNorm input (reads y2, dlogits)
  const int agrid = grid_for(nvox * 8, TPB);
  if (dtype == PCMS_BF16)
    launch_head_apply<bf16_t>(nt, agrid, s, y, dlogits, w, scale, shift, mean, invstd, coef, dy, nvox_per_n, N, ncls);
  else
    launch_head_apply<float>(nt, agrid, s, y, dlogits, w, scale, shift, mean, invstd, coef, dy, nvox_per_n, N, ncls);
  PCMS_CHECK_LAUNCH();
}

int pcms_loss_rows(long M) { return grid_for(M, TPB * 8, 1024); }

// loss (device fp32 scalar) and sums (device fp64[4]); part: rows*4 floats
int pcms_loss_fwd(const float* x, const float* t, long M, float smooth, float wb, float wd, float* part,
                  double* sums, float* loss, hipStream_t s) {
  const int rows = pcms_loss_rows(M);
  hipLaunchKernelGGL(loss_partial_kernel, dim3(rows), dim3(TPB), 0, s, x, t, M, part);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(loss_finalize_kernel, dim3(1), dim3(256), 0, s, (const float*)part, rows, M, smooth, wb, wd, sums, loss);
  PCMS_CHECK_LAUNCH();
}

int pcms_loss_bwd(const float* x, const float* t, long M, const double* sums, float smooth, float wb, float wd,
                  const float* gout, float* dx, hipStream_t s) {
  hipLaunchKernelGGL(loss_bwd_kernel, dim3(grid_for(M, TPB)), dim3(TPB), 0, s, x, t, M, sums, smooth, wb, wd, gout, dx);
  PCMS_CHECK_LAUNCH();
}

// step_size = lr / (1 - beta1^step), bc2_sqrt = sqrt(1 - beta2^step)  (host fp64 -> fp32)
int pcms_adam(float* p, float* g, float* m, float* v, long n, float step_size, float b1, float b2, float eps,
              float wd, float bc2_sqrt, float gscale, const float* gmul, hipStream_t s) {
  const AdamCoef c{step_size, b1, b2, eps, wd, bc2_sqrt, gscale};
  hipLaunchKernelGGL(adam_kernel, dim3(grid_for(n, TPB, 16384)), dim3(TPB), 0, s, p, g, m, v, n, c, gmul);
  PCMS_CHECK_LAUNCH();
}

int pcms_adam_ranges(float* p, float* g, float* m, float* v, const long long* ranges, int nranges, long max_len,
                     float step_size, float b1, float b2, float eps, float wd, float bc2_sqrt, float gscale,
                     const float* gmul, hipStream_t s) {
  if (nranges <= 0) return 0;
  const AdamCoef c{step_size, b1, b2, eps, wd, bc2_sqrt, gscale};
  hipLaunchKernelGGL(adam_ranges_kernel, dim3(grid_for(max_len, TPB, 2048), nranges), dim3(TPB), 0, s, p, g, m, v,
                     ranges, c, gmul);
  PCMS_CHECK_LAUNCH();
}

int pcms_fill_ranges(float* p, const long long* ranges, int nranges, long max_len, float v, hipStream_t s) {
  if (nranges <= 0) return 0;
  hipLaunchKernelGGL(fill_ranges_kernel, dim3(grid_for(max_len, TPB, 1024), nranges), dim3(TPB), 0, s, p, ranges, v);
  PCMS_CHECK_LAUNCH();
}

int pcms_grad_clip_ws_doubles(void) { return kNormBlocks; }

int pcms_grad_clip(float* g, long n, float gscale, float max_norm, int apply, double* ws, float* norm_out,
                   float* mul_out, hipStream_t s) {
  if (ws == nullptr || mul_out == nullptr || ((uintptr_t)g & 15)) return -1;
  const int rows = grid_for(n / 4 + 1, TPB, kNormBlocks);
  hipLaunchKernelGGL(sumsq_kernel, dim3(rows), dim3(TPB), 0, s, (const float*)g, n, ws);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(clip_finalize_kernel, dim3(1), dim3(256), 0, s, (const double*)ws, rows, gscale, max_norm,
                     norm_out, mul_out);
  e = hipGetLastError();
  if (e != hipSuccess || !apply) return (int)e;
  hipLaunchKernelGGL(scale_kernel, dim3(grid_for(n, TPB, 16384)), dim3(TPB), 0, s, g, n, (const float*)mul_out);
  PCMS_CHECK_LAUNCH();
}

int pcms_split_epilogue_rows(long nvox) { return cdiv(nvox, 64); }

int pcms_split_epilogue(int dtype, const float* acc, int splits, const float* bias, void* y0, void* y1, int cy0,
                        float* stats, int C, long nvox, int flags, hipStream_t s) {
  if (C % 64 || splits < 1) return -1;
  if (flags & ~PCMS_CONV_RELU || (stats && flags)) return -8;
  const int relu = flags & PCMS_CONV_RELU;
  if (y1 == nullptr) cy0 = C;
  dim3 grid(cdiv(nvox, 64), C / 64);
  if (dtype == PCMS_BF16) hipLaunchKernelGGL(split_epilogue_kernel<bf16_t>, grid, dim3(kSeThreads), 0, s, acc, splits, bias, (bf16_t*)y0, (bf16_t*)y1, cy0, stats, C, nvox, relu);
  else hipLaunchKernelGGL(split_epilogue_kernel<float>, grid, dim3(kSeThreads), 0, s, acc, splits, bias, (float*)y0, (float*)y1, cy0, stats, C, nvox, relu);
  PCMS_CHECK_LAUNCH();
}

int pcms_unpack_output(int dtype, const void* in, float* out, int N, int C, int Cs, long V, hipStream_t s) {
  if (C > Cs) return -1;
  const int grid = grid_for((long)N * C * V, TPB);
  if (dtype == PCMS_BF16) hipLaunchKernelGGL(unpack_output_kernel<bf16_t>, dim3(grid), dim3(TPB), 0, s, (const bf16_t*)in, out, N, C, Cs, V);
  else hipLaunchKernelGGL(unpack_output_kernel<float>, dim3(grid), dim3(TPB), 0, s, (const float*)in, out, N, C, Cs, V);
  PCMS_CHECK_LAUNCH();
}

int pcms_add(int dtype, void* dst, const void* src, long n, hipStream_t s) {
  const int VEC = dtype == PCMS_BF16 ? 8 : 4;
  if (n % VEC) return -1;
  const long nvec = n / VEC;
  if (dtype == PCMS_BF16) hipLaunchKernelGGL(add_kernel<bf16_t>, dim3(grid_for(nvec, TPB)), dim3(TPB), 0, s, (bf16_t*)dst, (const bf16_t*)src, nvec);
  else hipLaunchKernelGGL(add_kernel<float>, dim3(grid_for(nvec, TPB)), dim3(TPB), 0, s, (float*)dst, (const float*)src, nvec);
  PCMS_CHECK_LAUNCH();
}

}  // extern "C"
