// Stem kernel experiments (test tooling, not product): candidate kernels and load/store
// microbenchmarks, built into tests/kexp/libstemexp.so next to a copy of the product stem
// kernels (the #include below), driven by tests/kexp/stem_exp.py.
#include "../../prostate-cancer-multimodal-segmentation_amd/csrc/stem.hip"

namespace {
constexpr int kSWT4 = 256;  // the 4-wave wgrad experiment kernels

// ---------------------------------------------------------------------------------------
// (1) wave-specialised stem forward: waves 0-3 compute (MFMA, one per SIMD), waves 4-7 move
// memory (halo LDS-DMA, 16-B stores of the bf16 output, BatchNorm partial sums).  Compute
// wave c owns the 4 M-tiles (128 voxels) [128 c, 128 c + 128) of each 512-voxel box; each
// finished tile (32 voxels x 64 channels bf16 = 4 KiB) goes into an LDS ring of RS slots
// (voxel-major rows), handed to memory wave c + 4 by LDS counters (prod / cons).
// ---------------------------------------------------------------------------------------
constexpr int kWsRS = 4;
constexpr int kWsTile = 32 * 128;
constexpr int kWsHaloBytes = kHaloMax * 16;
constexpr int kWsOffW = 2 * kWsHaloBytes;
constexpr int kWsOffRing = kWsOffW + kStemSteps * 64 * 16 * 2;
constexpr int kWsOffRed = kWsOffRing + 4 * kWsRS * kWsTile;
constexpr int kWsOffFlags = kWsOffRed + 4 * 64 * 3 * 4;
constexpr int kWsLds = kWsOffFlags + 64;
constexpr int kSpinMax = 1 << 22;  // bounded spins (a protocol bug must not hang the GPU)

__device__ __forceinline__ int lds_ld(const volatile int* p) { return *p; }

// MODE bit 0: memory waves skip the BN sums; bit 1: compute waves skip the MFMAs
template <int LBD, int LBH, int MODE = 0>
__global__ void __launch_bounds__(512, 1) stem_fwd_ws_kernel(Conv3Params p, int nbox, int mrows, uint32_t xbytes,
                                                             uint32_t ybytes, int* err) {
  constexpr int bd = 1 << LBD, bh = 1 << LBH, bw = 16;
  constexpr int HH = bh + 2, HW = bw + 2, HV = (bd + 2) * HH * HW;
  constexpr int NPM = (HV + 255) / 256;
  static_assert(HV <= kHaloMax, "halo fits");
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r_lane = lane & 31, hsel = lane >> 5;
  const int D = p.D, H = p.H, W = p.W;
  const bool cw = wave < 4;
  const int pair = cw ? wave : wave - 4;
  volatile int* prod = reinterpret_cast<volatile int*>(lds + kWsOffFlags);
  volatile int* cons = prod + 4;
  float* red = reinterpret_cast<float*>(lds + kWsOffRed);
  char* ring = lds + kWsOffRing + pair * kWsRS * kWsTile;
  // weights -> LDS (packed [14][64][16] bf16, 28 KiB), counters -> 0
  {
    const u32x4_t* wg = reinterpret_cast<const u32x4_t*>(p.w);
    u32x4_t* wl = reinterpret_cast<u32x4_t*>(lds + kWsOffW);
    for (int i = tid; i < kStemSteps * 64 * 16 * 2 / 16; i += 512) wl[i] = wg[i];
    if (tid < 8) prod[tid] = 0;
  }
  const auto xr = __builtin_amdgcn_make_buffer_rsrc((void*)p.x0, 0, xbytes, 0x00020000);
  const auto yr = __builtin_amdgcn_make_buffer_rsrc(p.y0, 0, ybytes, 0x00020000);
  auto origin = [&](int b, int& n, int& d0, int& h0, int& w0) {
    int q = b;
    const int bwi = q % p.nbw; q /= p.nbw;
    const int bhi = q % p.nbh; q /= p.nbh;
    const int bdi = q % p.nbd;
    n = q / p.nbd;
    d0 = bdi * bd; h0 = bhi * bh; w0 = bwi * bw;
  };
  // memory waves: halo staging pieces (256 threads)
  const int mt_ = tid - 256;
  int prel[NPM], pco[NPM];
#pragma unroll
  for (int i = 0; i < NPM; ++i) {
    const int hv = mt_ + i * 256;
    const int hw_ = hv % HW, t_ = hv / HW, hh_ = t_ % HH, hd_ = t_ / HH;
    prel[i] = (((hd_ - 1) * H + (hh_ - 1)) * W + (hw_ - 1)) * 16;
    pco[i] = (hv >= 0 && hv < HV) ? (hd_ | (hh_ << 8) | (hw_ << 16)) : -1;
  }
  auto stage = [&](int b, int buf) {
    int n, d0, h0, w0;
    origin(b, n, d0, h0, w0);
    const int base16 = ((((n * D + d0) * H + h0) * W) + w0) * 16;
    const bool inner = d0 >= 1 && d0 + bd < D && h0 >= 1 && h0 + bh < H && w0 >= 1 && w0 + bw < W;
#pragma unroll
    for (int i = 0; i < NPM; ++i) {
      if (pair * 64 + i * 256 >= HV) break;
      uint32_t voff = (uint32_t)(base16 + prel[i]);
      const int c = pco[i];
      if (c < 0) {
        voff = kOOB;
      } else if (!inner) {
        const int gd = d0 + (c & 255) - 1, gh = h0 + ((c >> 8) & 255) - 1, gw = w0 + (c >> 16) - 1;
        if ((unsigned)gd >= (unsigned)D || (unsigned)gh >= (unsigned)H || (unsigned)gw >= (unsigned)W) voff = kOOB;
      }
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (LDS_AS void*)(lds + buf * kWsHaloBytes + (pair * 64 + i * 256) * 16),
                                               16, voff, 0, 0, 0);
    }
  };
  // compute waves: bias, halo row bases of the 4 M-tiles
  float bias_l[2] = {0.f, 0.f};
  if (p.bias) { bias_l[0] = p.bias[2 * r_lane]; bias_l[1] = p.bias[2 * r_lane + 1]; }
  int hb16[4];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) {
    const int r = pair * 128 + mt * 32 + perm32(r_lane);
    const int rd = r >> (LBH + 4), rh = (r >> 4) & (bh - 1), rw = r & 15;
    hb16[mt] = ((rd * HH + rh) * HW + rw) * 16;
  }
  // memory-wave BN state: lane holds channels 8 q .. 8 q + 7 of voxels x = 8 j + (lane >> 3)
  const int q8 = lane & 7, xl = lane >> 3;
  float s1[8], s2[8], K[8];
  float cnt = 0.f;
  bool first = true;
#pragma unroll
  for (int c = 0; c < 8; ++c) { s1[c] = 0.f; s2[c] = 0.f; K[c] = 0.f; }

  int b = blockIdx.x;
  if (!cw && b < nbox) stage(b, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  int t = 0;  // this pair's tile sequence number
  for (int it = 0; b < nbox; b += gridDim.x, ++it) {
    __syncthreads();  // halo(b) landed; every compute wave is done with the other buffer
    if (cw) {
      const char* hl = lds + (it & 1) * kWsHaloBytes;
      const char* wl = lds + kWsOffW;
      int hs16 = hsel * 16;
      asm volatile("" : "+v"(hs16));
#pragma unroll 1
      for (int mt = 0; mt < 4; ++mt, ++t) {
        f32x16_t acc[2];
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int e = 0; e < 16; ++e) acc[j][e] = bias_l[j];
        auto load_a = [&](int st) {
          const int o0 = tap_off(2 * st, HH, HW), o1 = tap_off(2 * st + 1, HH, HW);
          return *reinterpret_cast<const s16x8_t*>(hl + hb16[mt] + o0 * 16 + hs16 * (o1 - o0));
        };
        auto load_b = [&](int st, int nt) {
          return *reinterpret_cast<const s16x8_t*>(wl + ((st * 64 + nt * 32 + r_lane) * 16 + hsel * 8) * 2);
        };
        s16x8_t ab[2], bb[2][2];
        ab[0] = load_a(0);
        bb[0][0] = load_b(0, 0);
        bb[0][1] = load_b(0, 1);
#pragma unroll
        for (int st = 0; st < kStemSteps; ++st) {
          if (MODE & 2) break;
          if (st + 1 < kStemSteps) {
            ab[(st + 1) & 1] = load_a(st + 1);
            bb[(st + 1) & 1][0] = load_b(st + 1, 0);
            bb[(st + 1) & 1][1] = load_b(st + 1, 1);
          }
          acc[0] = mfma(ab[st & 1], bb[st & 1][0], acc[0]);
          acc[1] = mfma(ab[st & 1], bb[st & 1][1], acc[1]);
        }
        // wait for a free ring slot, write the tile (voxel-major rows), publish it
        const int slot = t % kWsRS;
        for (int k = 0; k < kSpinMax && t - lds_ld(cons + pair) >= kWsRS; ++k) __builtin_amdgcn_s_sleep(1);
        char* tile = ring + slot * kWsTile;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int rr = (e & 3) + 8 * (e >> 2) + 4 * hsel;
          *reinterpret_cast<uint32_t*>(tile + perm32(rr) * 128 + r_lane * 4) = pack_bf16x2(acc[0][e], acc[1][e]);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (lane == 0) prod[pair] = t + 1;
      }
    } else {
      const int bn = b + gridDim.x;
      if (bn < nbox) stage(bn, (it + 1) & 1);
      int n, d0, h0, w0;
      origin(b, n, d0, h0, w0);
      const bool full = d0 + bd <= D && h0 + bh <= H && w0 + bw <= W;
#pragma unroll 1
      for (int mt = 0; mt < 4; ++mt, ++t) {
        int k = 0;
        for (; k < kSpinMax && lds_ld(prod + pair) <= t; ++k) __builtin_amdgcn_s_sleep(1);
        if (k == kSpinMax && lane == 0) atomicAdd(err, 1);
        const char* tile = ring + (t % kWsRS) * kWsTile;
        u32x4_t v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = *reinterpret_cast<const u32x4_t*>(tile + (8 * j + xl) * 128 + q8 * 16);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (lane == 0) cons[pair] = t + 1;
        // tile voxels: box rows r = 128 pair + 32 mt + x (x = 8 j + xl): w = x & 15
        const int r0 = pair * 128 + mt * 32;
        if (first) {  // per-channel shift: this wave's first voxel (lanes 0-7 hold x = 0)
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            const uint32_t wv = __shfl(v[0][c], q8, 64);
            K[2 * c] = __uint_as_float(wv << 16);
            K[2 * c + 1] = __uint_as_float(wv & 0xffff0000u);
          }
          first = false;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int r = r0 + 8 * j + xl;
          const int rd = r >> (LBH + 4), rh = (r >> 4) & (bh - 1), rw = r & 15;
          const bool valid = full || (d0 + rd < D && h0 + rh < H && w0 + rw < W);
          const uint32_t voff = valid ? (uint32_t)((((n * D + d0 + rd) * H + h0 + rh) * W + w0 + rw) * 128 + q8 * 16)
                                      : kOOB;
          __builtin_amdgcn_raw_buffer_store_b128(v[j], yr, voff, 0, 0);
          if (valid && !(MODE & 1)) {
            cnt += 1.f;
#pragma unroll
            for (int c = 0; c < 4; ++c) {
              const float lo = __uint_as_float(v[j][c] << 16) - K[2 * c];
              const float hi = __uint_as_float(v[j][c] & 0xffff0000u) - K[2 * c + 1];
              s1[2 * c] += lo; s2[2 * c] = fmaf(lo, lo, s2[2 * c]);
              s1[2 * c + 1] += hi; s2[2 * c + 1] = fmaf(hi, hi, s2[2 * c + 1]);
            }
          }
        }
      }
      asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // halo(bn): 16 stores issued after it
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (!p.stats) return;
  // memory waves: reduce the 8 lanes sharing q (xor over lane bits 3-5), then (S, M2, n) per
  // wave and channel; Chan merge over the 4 memory waves
  if (!cw) {
    float nw = cnt;
    nw += __shfl_xor(nw, 8, 64); nw += __shfl_xor(nw, 16, 64); nw += __shfl_xor(nw, 32, 64);
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      float a = s1[c], q2 = s2[c];
      a += __shfl_xor(a, 8, 64); a += __shfl_xor(a, 16, 64); a += __shfl_xor(a, 32, 64);
      q2 += __shfl_xor(q2, 8, 64); q2 += __shfl_xor(q2, 16, 64); q2 += __shfl_xor(q2, 32, 64);
      if (xl == 0) {
        float* rp = red + (pair * 64 + 8 * q8 + c) * 3;
        rp[0] = a + nw * K[c];
        rp[1] = nw > 0.f ? q2 - a * a / nw : 0.f;
        rp[2] = nw;
      }
    }
  }
  __syncthreads();
  if (tid < 64) {
    float S = 0.f, Nn = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) { S += red[(w * 64 + tid) * 3]; Nn += red[(w * 64 + tid) * 3 + 2]; }
    const float m = Nn > 0.f ? S / Nn : 0.f;
    float M2 = 0.f, sdd = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const float c = red[(w * 64 + tid) * 3 + 2];
      if (c > 0.f) {
        const float d = red[(w * 64 + tid) * 3] / c - m;
        M2 += red[(w * 64 + tid) * 3 + 1] + c * d * d;
        sdd += c * d;
      }
    }
    if (Nn > 0.f) M2 -= sdd * sdd / Nn;
    float* st = p.stats + ((long)blockIdx.x * 64 + tid) * 2;
    st[0] = S;
    st[1] = M2;
    float* cnts = p.stats + (long)mrows * 128;
    if (tid == 0) cnts[blockIdx.x] = Nn;
    for (int r = blockIdx.x + gridDim.x; r < mrows; r += gridDim.x) {
      p.stats[((long)r * 64 + tid) * 2] = 0.f;
      p.stats[((long)r * 64 + tid) * 2 + 1] = 0.f;
      if (tid == 0) cnts[r] = 0.f;
    }
  }
}

// ---------------------------------------------------------------------------------------
// (2) stem wgrad load-pipeline experiments: the product kernel's box stream with switches
// MODE bit 0: compute, bit 1: halo DMA, bit 2: per-box barrier (else per-wave waits only)
// ---------------------------------------------------------------------------------------
template <int BD, int NS, int MODE>
__global__ void __launch_bounds__(kSWT4, 1) wg_exp_kernel(const bf16_t* x, const bf16_t* dy, float* part,
                                                        int N, int D, int H, int W, uint32_t xbytes,
                                                        uint32_t dybytes) {
  typedef SWGeom<BD, kSWT4> Gm;
  constexpr bool COMP = MODE & 1, HALO = MODE & 2, BAR = MODE & 4;
  constexpr int BH = 4, BW = 16, HH = BH + 2, HW = BW + 2;
  constexpr int kSWBV = Gm::BV, kSWHV = Gm::HV, kSWBuf = Gm::Buf;
  constexpr int XI = HALO ? Gm::XI : 0;
  extern __shared__ __attribute__((aligned(16))) char swl[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hsel = lane >> 5;
  const int nbw = W / BW, nbh = H / BH, nbd = D / BD;
  const int nbox = N * nbd * nbh * nbw;
  const i32x4_t xr = buffer_desc(x, xbytes);
  const i32x4_t dr = buffer_desc(dy, dybytes);
  uint32_t dyrel[Gm::DYP];
#pragma unroll
  for (int i = 0; i < Gm::DYP; ++i) {
    const int pc = tid + i * kSWT4;
    const int r = pc >> 3, q = pc & 7;
    const int ql = q ^ (((r >> 1) & 1) << 2);
    const int rd = r >> 6, rh = (r >> 4) & 3, rw = r & 15;
    dyrel[i] = (uint32_t)(((rd * H + rh) * W + rw) * 128 + ql * 16);
  }
  const int nxp = HALO ? (Gm::HRows / 64 - wave + 3) / 4 : 0;
  int xrel[Gm::XI], xco[Gm::XI];
#pragma unroll
  for (int i = 0; i < Gm::XI; ++i) {
    const int hv = wave * 64 + lane + i * kSWT4;
    const int hw_ = hv % HW, t_ = hv / HW, hh_ = t_ % HH, hd_ = t_ / HH;
    xrel[i] = (((hd_ - 1) * H + (hh_ - 1)) * W + (hw_ - 1)) * 16;
    xco[i] = hv < kSWHV ? (hd_ | (hh_ << 8) | (hw_ << 16)) : -1;
  }
  auto origin = [&](int b, int& n, int& d0, int& h0, int& w0) {
    int q = b;
    const int bwi = q % nbw; q /= nbw;
    const int bhi = q % nbh; q /= nbh;
    const int bdi = q % nbd;
    n = q / nbd;
    d0 = bdi * BD; h0 = bhi * BH; w0 = bwi * BW;
  };
  auto stage = [&](int b, int slot) {
    int n, d0, h0, w0;
    origin(b, n, d0, h0, w0);
    const int vb = ((n * D + d0) * H + h0) * W + w0;
    const uint32_t lb = __builtin_amdgcn_readfirstlane(lds_addr(swl) + slot * kSWBuf + wave * 64 * 16);
    const uint32_t so = __builtin_amdgcn_readfirstlane((uint32_t)vb * 128u);
#pragma unroll
    for (int i = 0; i < Gm::DYP; ++i) dma16(dr, lb + i * kSWT4 * 16, dyrel[i], so);
    const bool inner = d0 >= 1 && d0 + BD < D && h0 >= 1 && h0 + BH < H && w0 >= 1 && w0 + BW < W;
#pragma unroll
    for (int i = 0; i < XI; ++i) {
      if (i >= nxp) break;
      uint32_t voff = (uint32_t)(vb * 16 + xrel[i]);
      const int c = xco[i];
      if (c < 0) {
        voff = kOOB;
      } else if (!inner) {
        const int gd = d0 + (c & 255) - 1, gh = h0 + ((c >> 8) & 255) - 1, gw = w0 + (c >> 16) - 1;
        if ((unsigned)gd >= (unsigned)D || (unsigned)gh >= (unsigned)H || (unsigned)gw >= (unsigned)W) voff = kOOB;
      }
      dma16(xr, lb + kSWBV * 128 + i * kSWT4 * 16, voff, 0);
    }
  };
  const int g = (lane >> 4) & 1, qq = (lane & 15) >> 2, pp = lane & 3;
  f32x16_t acc[2][7];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 7; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
  const int aoff0 = dy_off_bf16(8 * hsel + qq, g * 16 + pp * 4) + wave * 2048;
  const int aoff1 = dy_off_bf16(8 * hsel + qq, 32 + g * 16 + pp * 4) + wave * 2048;
  int boff[7];
#pragma unroll
  for (int j = 0; j < 7; ++j)
    boff[j] = kSWBV * 128 + (8 * hsel + qq + tap_off(4 * j + 2 * g + (pp >> 1), HH, HW) + wave * HW) * 16 + (pp & 1) * 8;
  auto compute = [&](const char* buf) {
    uint32_t pa0 = lds_addr(buf) + aoff0, pa1 = lds_addr(buf) + aoff1, pb[7];
#pragma unroll
    for (int j = 0; j < 7; ++j) pb[j] = lds_addr(buf) + boff[j];
    asm volatile("" : "+v"(pa0), "+v"(pa1), "+v"(pb[0]), "+v"(pb[1]), "+v"(pb[2]), "+v"(pb[3]), "+v"(pb[4]),
                 "+v"(pb[5]), "+v"(pb[6]));
    auto tr = [](uint32_t p, int off) {
      return __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4_t*)(uintptr_t)(p + off));
    };
    auto cat = [](s16x4_t lo, s16x4_t hi) { return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7); };
    auto load = [&](int i, s16x8_t (&a)[2], s16x8_t (&bq)[7]) {
      const int dyb = i * 4 * 2048;
      const int hrb = i * HH * HW * 16;
      a[0] = cat(tr(pa0, dyb), tr(pa0, dyb + 512));
      a[1] = cat(tr(pa1, dyb), tr(pa1, dyb + 512));
#pragma unroll
      for (int j = 0; j < 7; ++j) bq[j] = cat(tr(pb[j], hrb), tr(pb[j], hrb + 64));
    };
    s16x8_t a[2][2], bq[2][7];
    load(0, a[0], bq[0]);
#pragma unroll
    for (int i = 0; i < BD; ++i) {
      if (i + 1 < BD) load(i + 1, a[(i + 1) & 1], bq[(i + 1) & 1]);
#pragma unroll
      for (int j = 0; j < 7; ++j)
#pragma unroll
        for (int ct = 0; ct < 2; ++ct) acc[ct][j] = mfma(a[i & 1][ct], bq[i & 1][j], acc[ct][j]);
    }
  };
  const int G = gridDim.x;
  int b = blockIdx.x;
#pragma unroll
  for (int k = 0; k < NS - 1; ++k)
    if (b + k * G < nbox) stage(b + k * G, k);
  constexpr int PER = Gm::DYP + XI;
  for (int it = 0; b < nbox; b += G, ++it) {
    if (b + (NS - 2) * G < nbox) {
      if (!HALO || nxp == Gm::XI) asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NS - 2) * PER) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NS - 2) * (PER - 1)) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    if constexpr (BAR) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
    const int b2 = b + (NS - 1) * G;
    if (b2 < nbox) stage(b2, (it + NS - 1) % NS);
    if constexpr (COMP) compute(swl + (it % NS) * kSWBuf);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  // keep the accumulators live
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 7; ++j) s += acc[i][j][0];
  if (s == 12345.f) part[tid] = s;
}

// plain streaming reads of the same dy bytes by global_load_dwordx4 (no LDS), 8 waves per CU
__global__ void __launch_bounds__(512) read_stream_kernel(const u32x4_t* y, long n16, float* out) {
  uint32_t s = 0;
  for (long i = blockIdx.x * 512L + threadIdx.x; i < n16; i += (long)gridDim.x * 512) {
    const u32x4_t v = y[i];
    s ^= v.x + v.y + v.z + v.w;
  }
  if (s == 0x12345678u) out[0] = 1.f;
}


// ---------------------------------------------------------------------------------------
// (3) stem forward v3: the direct kernel with (a) 16-B stores: a DPP 4x4 transpose inside
// each lane quad turns 4 channel-pair dwords x 4 voxel rows into one voxel's 8 channels per
// lane, so a store instruction writes two 512-B runs (8 per box and wave instead of 32
// dword stores), and (b) a 3-buffer halo ring prefetched two boxes ahead, so a wave only
// ever waits for stores two boxes old (vmcnt counts stores and loads in one queue).  Every
// wave issues exactly NP DMA pieces and 8 stores per box (out-of-range ones are dropped),
// so the vmcnt values are constants.
// ---------------------------------------------------------------------------------------
// lane exchange inside a quad (lane ^ M) through the LDS crossbar (ds_swizzle, quad mode):
// a DPP move here was corrupted in about 1e-4 of the dwords on gfx950 (an unchecked hazard)
template <int M> __device__ __forceinline__ uint32_t dpp_xor(uint32_t v) {
  // ds_swizzle offset: bit 15 = quad-permute mode, bits [7:0] = 4 x 2-bit lane selects
  constexpr int pat = 0x8000 | (M == 1 ? 0xB1 : 0x4E);
  return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, pat);
}
// lane j = lane & 3 of a quad holds v[i] = M[j][i]; afterwards v[i] = M[i][j]
__device__ __forceinline__ void quad_transpose(uint32_t (&v)[4], int j) {
  {
    const bool hi = j & 1;
    uint32_t a = hi ? v[0] : v[1], c = hi ? v[2] : v[3];
    a = dpp_xor<1>(a);
    c = dpp_xor<1>(c);
    if (hi) { v[0] = a; v[2] = c; } else { v[1] = a; v[3] = c; }
  }
  {
    const bool hi = j & 2;
    uint32_t a = hi ? v[0] : v[2], c = hi ? v[1] : v[3];
    a = dpp_xor<2>(a);
    c = dpp_xor<2>(c);
    if (hi) { v[0] = a; v[1] = c; } else { v[2] = a; v[3] = c; }
  }
}

constexpr int kS3NP = 3;                          // DMA pieces per thread and box (fixed)
constexpr int kS3Buf = kS3NP * 512 * 16;          // 24 KiB per halo buffer
constexpr int kS3W = 3 * kS3Buf;                  // packed weights [14][64][32 B] (28 KiB)
constexpr int kS3T = kS3W + kStemSteps * 64 * 32;  // transpose scratch: 8 waves x [4][64] dwords
constexpr int kS3Lds = kS3T + 8 * 1024 + 8 * 64 * 3 * 4;

// MODE bit 0: no stores, bit 1: no MFMA, bit 2: no epilogue VALU (BN sums, pack, transpose)
template <int LBD, int LBH, int MODE = 0>
__global__ void __launch_bounds__(512, 1) stem_fwd_v3_kernel(Conv3Params p, int nbox, int mrows, uint32_t xbytes,
                                                             uint32_t ybytes) {
  constexpr int NWV = 8;
  constexpr int bd = 1 << LBD, bh = 1 << LBH, bw = 16;
  constexpr int HH = bh + 2, HW = bw + 2, HV = (bd + 2) * HH * HW;
  static_assert(HV <= kS3NP * 512, "halo fits the fixed piece count");
  static_assert((1 << (LBD + LBH + 4)) == NWV * 64, "box = 64 voxels per wave");
  extern __shared__ __attribute__((aligned(16))) char lds[];
  float* red = reinterpret_cast<float*>(lds + kS3T + 8 * 1024);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r_lane = lane & 31, hsel = lane >> 5;
  const int D = p.D, H = p.H, W = p.W;
  const int G = gridDim.x;
  const i32x4_t xr = buffer_desc(p.x0, xbytes);
  const auto yr = __builtin_amdgcn_make_buffer_rsrc(p.y0, 0, ybytes, 0x00020000);
  // weights -> LDS once: row (st, col) 32 B, its two 16-B k-halves swapped when col bit 4 is
  // set (the ds_read_b128 lane groups then cover all 64 banks)
  {
    const u32x4_t* wg = reinterpret_cast<const u32x4_t*>(p.w);
    for (int i = tid; i < kStemSteps * 64 * 2; i += 512) {
      const int row = i >> 1, half = i & 1, col = row & 63;
      *reinterpret_cast<u32x4_t*>(lds + kS3W + row * 32 + ((half ^ ((col >> 4) & 1)) * 16)) = wg[i];
    }
  }
  const int wrow = (r_lane * 32) + ((hsel ^ ((r_lane >> 4) & 1)) * 16);  // + (st * 64 + 32 nt) * 32
  float bias_l[2] = {0.f, 0.f};
  if (p.bias) { bias_l[0] = p.bias[2 * r_lane]; bias_l[1] = p.bias[2 * r_lane + 1]; }
  int hb16[2];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) {
    const int r = wave * 64 + mt * 32 + perm32(r_lane);
    const int rd = r >> (LBH + 4), rh = (r >> 4) & (bh - 1), rw = r & 15;
    hb16[mt] = ((rd * HH + rh) * HW + rw) * 16;
  }
  int prel[kS3NP], pco[kS3NP];
#pragma unroll
  for (int i = 0; i < kS3NP; ++i) {
    const int hv = tid + i * 512;
    const int hw_ = hv % HW, t_ = hv / HW, hh_ = t_ % HH, hd_ = t_ / HH;
    prel[i] = (((hd_ - 1) * H + (hh_ - 1)) * W + (hw_ - 1)) * 16;
    pco[i] = hv < HV ? (hd_ | (hh_ << 8) | (hw_ << 16)) : -1;
  }
  // store lanes: quad kq (channels 8 kq .. 8 kq + 7), j = row within the quad's 4 rows
  const int j = lane & 3, kq = r_lane >> 2;
  uint32_t voffg[4];
  int xg[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int x = perm32(8 * g + 4 * hsel) + j;  // tile voxel: h-row x >> 4, w x & 15
    xg[g] = x;
    voffg[g] = (uint32_t)(((x >> 4) * W + (x & 15)) * 128 + kq * 16);
  }
  auto origin = [&](int b, int& n, int& d0, int& h0, int& w0) {
    int q = b;
    const int bwi = q % p.nbw; q /= p.nbw;
    const int bhi = q % p.nbh; q /= p.nbh;
    const int bdi = q % p.nbd;
    n = q / p.nbd;
    d0 = bdi * bd; h0 = bhi * bh; w0 = bwi * bw;
  };
  // always kS3NP pieces (a box past the end: every piece out of range -> zeros)
  auto stage = [&](int b, int buf) {
    if (MODE & 8) return;
    int n = 0, d0 = 0, h0 = 0, w0 = 0;
    const bool live = b < nbox;
    if (live) origin(b, n, d0, h0, w0);
    const int base16 = ((((n * D + d0) * H + h0) * W) + w0) * 16;
    const bool inner = d0 >= 1 && d0 + bd < D && h0 >= 1 && h0 + bh < H && w0 >= 1 && w0 + bw < W;
#pragma unroll
    for (int i = 0; i < kS3NP; ++i) {
      uint32_t voff = (uint32_t)(base16 + prel[i]);
      const int c = pco[i];
      if (c < 0 || !live) {
        voff = kOOB;
      } else if (!inner) {
        const int gd = d0 + (c & 255) - 1, gh = h0 + ((c >> 8) & 255) - 1, gw = w0 + (c >> 16) - 1;
        if ((unsigned)gd >= (unsigned)D || (unsigned)gh >= (unsigned)H || (unsigned)gw >= (unsigned)W) voff = kOOB;
      }
      // inline-asm DMA (see dma16): the compiler's waitcnt pass would otherwise drain vmcnt
      // -- this wave's in-flight stores included -- before every LDS read of the halo
      dma16(xr, __builtin_amdgcn_readfirstlane(lds_addr(lds + buf * kS3Buf + (wave * 64 + i * 512) * 16)), voff, 0);
    }
  };
  float s1[2] = {0.f, 0.f}, s2[2] = {0.f, 0.f}, K[2] = {0.f, 0.f};
  float cnt = 0.f;
  bool first = true;
  int b = blockIdx.x;
  stage(b, 0);
  stage(b + G, 1);
  for (int it = 0; b < nbox; b += G, ++it) {
    // halo(b) landed: the ops this wave issued after its DMA are the next box's DMA and the
    // stores of the (up to) two boxes before this one
    if (MODE & 8) {
      asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    } else if (it == 0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kS3NP) : "memory");
    else if (it == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kS3NP + 8) : "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kS3NP + 16) : "memory");
    if (!(MODE & 16)) __syncthreads();
    stage(b + 2 * G, (it + 2) % 3);
    const char* hl = lds + (it % 3) * kS3Buf;
    f32x16_t acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[i][jj][e] = bias_l[jj];
    {
      int hs16 = hsel * 16;
      asm volatile("" : "+v"(hs16));
      auto load_a = [&](int st, s16x8_t (&a)[2]) {
        const int o0 = tap_off(2 * st, HH, HW), o1 = tap_off(2 * st + 1, HH, HW);
        const int off16 = o0 * 16 + hs16 * (o1 - o0);
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) a[mt] = *reinterpret_cast<const s16x8_t*>(hl + hb16[mt] + off16);
      };
      const char* wl = lds + kS3W + wrow;
      auto load_b = [&](int st, s16x8_t (&w)[2]) {
        w[0] = *reinterpret_cast<const s16x8_t*>(wl + st * 64 * 32);
        w[1] = *reinterpret_cast<const s16x8_t*>(wl + (st * 64 + 32) * 32);
      };
      s16x8_t abuf[2][2], bbuf[2][2];
      load_a(0, abuf[0]);
      load_b(0, bbuf[0]);
#pragma unroll
      for (int st = 0; st < kStemSteps; ++st) {
        if (MODE & 2) break;
        if (st + 1 < kStemSteps) {
          load_a(st + 1, abuf[(st + 1) & 1]);
          load_b(st + 1, bbuf[(st + 1) & 1]);
        }
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
          acc[mt][0] = mfma(abuf[st & 1][mt], bbuf[st & 1][0], acc[mt][0]);
          acc[mt][1] = mfma(abuf[st & 1][mt], bbuf[st & 1][1], acc[mt][1]);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    int n, d0, h0, w0;
    origin(b, n, d0, h0, w0);
    const bool full = d0 + bd <= D && h0 + bh <= H && w0 + bw <= W;
    if (first) {
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) K[nt] = __shfl(acc[0][nt][0], r_lane, 64);
      first = false;
    }
    const int bv = ((n * D + d0) * H + h0) * W + w0;
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      const int R0 = wave * 4 + mt * 2;
      const int rd0 = R0 >> LBH, rh0 = R0 & (bh - 1);
      const uint32_t so = __builtin_amdgcn_readfirstlane((uint32_t)(bv + (rd0 * H + rh0) * W) * 128u);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        if ((MODE & 4) && g > 0) break;
        uint32_t v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int e = 4 * g + i;
          const float v0 = acc[mt][0][e], v1 = acc[mt][1][e];
          v[i] = pack_bf16x2(v0, v1);
          float e0 = v0 - K[0], e1 = v1 - K[1];
          if (!full) {
            const int x = perm32((e & 3) + 8 * (e >> 2) + 4 * hsel);
            const bool valid = (d0 + rd0 < D) & (h0 + rh0 + (x >> 4) < H) & (w0 + (x & 15) < W);
            e0 = valid ? e0 : 0.f;
            e1 = valid ? e1 : 0.f;
            cnt += valid ? 1.f : 0.f;
          }
          s1[0] += e0; s2[0] = fmaf(e0, e0, s2[0]);
          s1[1] += e1; s2[1] = fmaf(e1, e1, s2[1]);
        }
        // 4x4 transpose inside each lane quad through this wave's LDS scratch [i][lane]
        {
          uint32_t* tw = reinterpret_cast<uint32_t*>(lds + kS3T + wave * 1024);
#pragma unroll
          for (int i = 0; i < 4; ++i) tw[i * 64 + lane] = v[i];
          const u32x4_t t4 = *reinterpret_cast<const u32x4_t*>(tw + j * 64 + (lane & ~3));
          v[0] = t4[0]; v[1] = t4[1]; v[2] = t4[2]; v[3] = t4[3];
        }
        uint32_t voff = voffg[g];
        if (!full) {
          const int x = xg[g];
          const bool valid = (d0 + rd0 < D) & (h0 + rh0 + (x >> 4) < H) & (w0 + (x & 15) < W);
          voff = valid ? voff : kOOB;
        }
        const u32x4_t q4 = {v[0], v[1], v[2], v[3]};
        if (!(MODE & 1)) {
          if (MODE & 32) {  // the same bytes as whole contiguous 1-KiB pieces (a 64-KiB slab per box)
#pragma unroll
            for (int gg = 0; gg < 4; ++gg)
              __builtin_amdgcn_raw_buffer_store_b128(q4, yr, (uint32_t)(lane * 16 + gg * 1024 + mt * 4096),
                                                     __builtin_amdgcn_readfirstlane((uint32_t)b * 65536u + wave * 8192u), 0);
          } else if (MODE & 4) {  // the four stores of the group without its epilogue work
#pragma unroll
            for (int gg = 0; gg < 4; ++gg) __builtin_amdgcn_raw_buffer_store_b128(q4, yr, voffg[gg], so, 0);
          } else {
            __builtin_amdgcn_raw_buffer_store_b128(q4, yr, voff, so, 0);
          }
        }
      }
    }
    if (full) cnt += 32.f;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (!p.stats) return;
  const float nw = cnt + __shfl_xor(cnt, 32, 64);
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) {
    s1[nt] += __shfl_xor(s1[nt], 32, 64);
    s2[nt] += __shfl_xor(s2[nt], 32, 64);
    if (hsel == 0) {
      float* rp = red + (wave * 64 + 2 * r_lane + nt) * 3;
      rp[0] = s1[nt] + nw * K[nt];
      rp[1] = nw > 0.f ? s2[nt] - s1[nt] * s1[nt] / nw : 0.f;
      rp[2] = nw;
    }
  }
  __syncthreads();
  if (tid < 64) {
    float S = 0.f, Nn = 0.f;
#pragma unroll
    for (int w = 0; w < NWV; ++w) { S += red[(w * 64 + tid) * 3]; Nn += red[(w * 64 + tid) * 3 + 2]; }
    const float m = Nn > 0.f ? S / Nn : 0.f;
    float M2 = 0.f, sdd = 0.f;
#pragma unroll
    for (int w = 0; w < NWV; ++w) {
      const float c = red[(w * 64 + tid) * 3 + 2];
      if (c > 0.f) {
        const float d = red[(w * 64 + tid) * 3] / c - m;
        M2 += red[(w * 64 + tid) * 3 + 1] + c * d * d;
        sdd += c * d;
      }
    }
    if (Nn > 0.f) M2 -= sdd * sdd / Nn;
    float* st = p.stats + ((long)blockIdx.x * 64 + tid) * 2;
    st[0] = S;
    st[1] = M2;
    float* cnts = p.stats + (long)mrows * 128;
    if (tid == 0) cnts[blockIdx.x] = Nn;
    for (int r = blockIdx.x + gridDim.x; r < mrows; r += gridDim.x) {
      p.stats[((long)r * 64 + tid) * 2] = 0.f;
      p.stats[((long)r * 64 + tid) * 2 + 1] = 0.f;
      if (tid == 0) cnts[r] = 0.f;
    }
  }
}

// ---------------------------------------------------------------------------------------
// (4) stem wgrad v2: the product stream kernel with a two-stage LDS flush (waves 0/1 write
// their 14 tiles lane-major into two regions, waves 2/3 add theirs, then every thread sums
// the two regions into the partial row) instead of four serial read-modify-write passes
// ---------------------------------------------------------------------------------------
constexpr int kW2LaneStride = 20;                        // floats per lane (16 used, conflict-free b128)
constexpr int kW2Region = 14 * 64 * kW2LaneStride * 4;   // 71,680 B
constexpr int kW2Lds = kSWRing > 2 * kW2Region ? kSWRing : 2 * kW2Region;

template <int BD, int NS>
__global__ void __launch_bounds__(kSWT4, 1) stem_wgrad_v2_kernel(const bf16_t* x, const bf16_t* dy, float* part,
                                                               int N, int D, int H, int W, int cin_w,
                                                               uint32_t xbytes, uint32_t dybytes) {
  typedef SWGeom<BD, kSWT4> Gm;
  constexpr int BH = 4, BW = 16, HH = BH + 2, HW = BW + 2;
  constexpr int kSWBV = Gm::BV, kSWHV = Gm::HV, kSWBuf = Gm::Buf;
  extern __shared__ __attribute__((aligned(16))) char swl[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hsel = lane >> 5;
  const int nbw = W / BW, nbh = H / BH, nbd = D / BD;
  const int nbox = N * nbd * nbh * nbw;
  const i32x4_t xr = buffer_desc(x, xbytes);
  const i32x4_t dr = buffer_desc(dy, dybytes);
  uint32_t dyrel[Gm::DYP];
#pragma unroll
  for (int i = 0; i < Gm::DYP; ++i) {
    const int pc = tid + i * kSWT4;
    const int r = pc >> 3, q = pc & 7;
    const int ql = q ^ (((r >> 1) & 1) << 2);
    const int rd = r >> 6, rh = (r >> 4) & 3, rw = r & 15;
    dyrel[i] = (uint32_t)(((rd * H + rh) * W + rw) * 128 + ql * 16);
  }
  const int nxp = (Gm::HRows / 64 - wave + 3) / 4;
  int xrel[Gm::XI], xco[Gm::XI];
#pragma unroll
  for (int i = 0; i < Gm::XI; ++i) {
    const int hv = wave * 64 + lane + i * kSWT4;
    const int hw_ = hv % HW, t_ = hv / HW, hh_ = t_ % HH, hd_ = t_ / HH;
    xrel[i] = (((hd_ - 1) * H + (hh_ - 1)) * W + (hw_ - 1)) * 16;
    xco[i] = hv < kSWHV ? (hd_ | (hh_ << 8) | (hw_ << 16)) : -1;
  }
  auto origin = [&](int b, int& n, int& d0, int& h0, int& w0) {
    int q = b;
    const int bwi = q % nbw; q /= nbw;
    const int bhi = q % nbh; q /= nbh;
    const int bdi = q % nbd;
    n = q / nbd;
    d0 = bdi * BD; h0 = bhi * BH; w0 = bwi * BW;
  };
  auto stage = [&](int b, int slot) {
    int n, d0, h0, w0;
    origin(b, n, d0, h0, w0);
    const int vb = ((n * D + d0) * H + h0) * W + w0;
    const uint32_t lb = __builtin_amdgcn_readfirstlane(lds_addr(swl) + slot * kSWBuf + wave * 64 * 16);
    const uint32_t so = __builtin_amdgcn_readfirstlane((uint32_t)vb * 128u);
#pragma unroll
    for (int i = 0; i < Gm::DYP; ++i) dma16(dr, lb + i * kSWT4 * 16, dyrel[i], so);
    const bool inner = d0 >= 1 && d0 + BD < D && h0 >= 1 && h0 + BH < H && w0 >= 1 && w0 + BW < W;
#pragma unroll
    for (int i = 0; i < Gm::XI; ++i) {
      if (i >= nxp) break;
      uint32_t voff = (uint32_t)(vb * 16 + xrel[i]);
      const int c = xco[i];
      if (c < 0) {
        voff = kOOB;
      } else if (!inner) {
        const int gd = d0 + (c & 255) - 1, gh = h0 + ((c >> 8) & 255) - 1, gw = w0 + (c >> 16) - 1;
        if ((unsigned)gd >= (unsigned)D || (unsigned)gh >= (unsigned)H || (unsigned)gw >= (unsigned)W) voff = kOOB;
      }
      dma16(xr, lb + kSWBV * 128 + i * kSWT4 * 16, voff, 0);
    }
  };
  const int g = (lane >> 4) & 1, qq = (lane & 15) >> 2, pp = lane & 3;
  f32x16_t acc[2][7];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int jj = 0; jj < 7; ++jj)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][jj][e] = 0.f;
  const int aoff0 = dy_off_bf16(8 * hsel + qq, g * 16 + pp * 4) + wave * 2048;
  const int aoff1 = dy_off_bf16(8 * hsel + qq, 32 + g * 16 + pp * 4) + wave * 2048;
  int boff[7];
#pragma unroll
  for (int jj = 0; jj < 7; ++jj)
    boff[jj] = kSWBV * 128 + (8 * hsel + qq + tap_off(4 * jj + 2 * g + (pp >> 1), HH, HW) + wave * HW) * 16 + (pp & 1) * 8;
  auto compute = [&](const char* buf) {
    uint32_t pa0 = lds_addr(buf) + aoff0, pa1 = lds_addr(buf) + aoff1, pb[7];
#pragma unroll
    for (int jj = 0; jj < 7; ++jj) pb[jj] = lds_addr(buf) + boff[jj];
    asm volatile("" : "+v"(pa0), "+v"(pa1), "+v"(pb[0]), "+v"(pb[1]), "+v"(pb[2]), "+v"(pb[3]), "+v"(pb[4]),
                 "+v"(pb[5]), "+v"(pb[6]));
    auto tr = [](uint32_t p, int off) {
      return __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4_t*)(uintptr_t)(p + off));
    };
    auto cat = [](s16x4_t lo, s16x4_t hi) { return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7); };
    auto load = [&](int i, s16x8_t (&a)[2], s16x8_t (&bq)[7]) {
      const int dyb = i * 4 * 2048;
      const int hrb = i * HH * HW * 16;
      a[0] = cat(tr(pa0, dyb), tr(pa0, dyb + 512));
      a[1] = cat(tr(pa1, dyb), tr(pa1, dyb + 512));
#pragma unroll
      for (int jj = 0; jj < 7; ++jj) bq[jj] = cat(tr(pb[jj], hrb), tr(pb[jj], hrb + 64));
    };
    s16x8_t a[2][2], bq[2][7];
    load(0, a[0], bq[0]);
#pragma unroll
    for (int i = 0; i < BD; ++i) {
      if (i + 1 < BD) load(i + 1, a[(i + 1) & 1], bq[(i + 1) & 1]);
#pragma unroll
      for (int jj = 0; jj < 7; ++jj)
#pragma unroll
        for (int ct = 0; ct < 2; ++ct) acc[ct][jj] = mfma(a[i & 1][ct], bq[i & 1][jj], acc[ct][jj]);
    }
  };
  const int G = gridDim.x;
  int b = blockIdx.x;
#pragma unroll
  for (int k = 0; k < NS - 1; ++k)
    if (b + k * G < nbox) stage(b + k * G, k);
  for (int it = 0; b < nbox; b += G, ++it) {
    if (b + (NS - 2) * G < nbox) {
      if (nxp == Gm::XI) asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NS - 2) * (Gm::DYP + Gm::XI)) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NS - 2) * (Gm::DYP + Gm::XI - 1)) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    const int b2 = b + (NS - 1) * G;
    if (b2 < nbox) stage(b2, (it + NS - 1) % NS);
    compute(swl + (it % NS) * kSWBuf);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // flush: region (wave & 1); waves 0/1 store, waves 2/3 add; tile t = ct * 7 + jj, lane-major
  float* reg = reinterpret_cast<float*>(swl) + (wave & 1) * (kW2Region / 4);
  if (wave < 2) {
#pragma unroll
    for (int ct = 0; ct < 2; ++ct)
#pragma unroll
      for (int jj = 0; jj < 7; ++jj) {
        float* dst = reg + ((ct * 7 + jj) * 64 + lane) * kW2LaneStride;
#pragma unroll
        for (int q = 0; q < 4; ++q)
          *reinterpret_cast<f32x4_t*>(dst + 4 * q) = (f32x4_t){acc[ct][jj][4 * q], acc[ct][jj][4 * q + 1],
                                                                acc[ct][jj][4 * q + 2], acc[ct][jj][4 * q + 3]};
      }
  }
  __syncthreads();
  if (wave >= 2) {
#pragma unroll
    for (int ct = 0; ct < 2; ++ct)
#pragma unroll
      for (int jj = 0; jj < 7; ++jj) {
        float* dst = reg + ((ct * 7 + jj) * 64 + lane) * kW2LaneStride;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          f32x4_t v = *reinterpret_cast<f32x4_t*>(dst + 4 * q);
          v += (f32x4_t){acc[ct][jj][4 * q], acc[ct][jj][4 * q + 1], acc[ct][jj][4 * q + 2], acc[ct][jj][4 * q + 3]};
          *reinterpret_cast<f32x4_t*>(dst + 4 * q) = v;
        }
      }
  }
  __syncthreads();
  // partial row [64 co][cin_w][27]: value (co, col = 8 t + c) lives in tile (co >> 5, col >> 5), lane
  // (col & 31) + 32 hs, element e with (e & 3) + 8 (e >> 2) + 4 hs = co & 31
  const float* r0 = reinterpret_cast<const float*>(swl);
  const float* r1 = r0 + kW2Region / 4;
  const int per_co = cin_w * 27;
  const int total = 64 * per_co;
  float* prow = part + (long)blockIdx.x * total;
  for (int i = tid; i < total; i += kSWT4) {
    const int co = i / per_co, rem = i - co * per_co;
    const int c = rem / 27, t = rem - c * 27;
    const int col = 8 * t + c;
    const int cr = co & 31, hs = (cr >> 2) & 1, e = (cr & 3) + 4 * (cr >> 3);
    const int off = (((co >> 5) * 7 + (col >> 5)) * 64 + (col & 31) + 32 * hs) * kW2LaneStride + e;
    prow[i] = r0[off] + r1[off];
  }
}

}  // namespace

extern "C" {

int exp_stem_fwd_ws(int mode, const void* x, const void* wpack, const float* bias, void* y, float* stats, int* err,
                    int N, int D, int H, int W, hipStream_t s) {
  const Box b = fwd_box(D, H, W);
  if (!(b.lbw == 4 && b.lbd + b.lbh == 5 && (b.lbd == 2 || b.lbd == 3))) return -5;
  Conv3Params p;
  p.x0 = x; p.x1 = nullptr; p.c0 = 8; p.c1 = 0;
  p.w = wpack; p.bias = bias; p.y0 = y; p.y1 = nullptr; p.cy0 = 64;
  p.yacc = nullptr; p.stats = stats; p.accumulate = 0;
  p.N = N; p.D = D; p.H = H; p.W = W; p.Cin = 8; p.Cout = 64;
  p.nvox = (long)N * D * H * W;
  p.nchunk = 1; p.chunks_per_split = 1;
  p.lbd = b.lbd; p.lbh = b.lbh; p.lbw = b.lbw;
  p.nbd = cdiv(D, 1 << b.lbd); p.nbh = cdiv(H, 1 << b.lbh); p.nbw = cdiv(W, 1 << b.lbw);
  const int nbox = N * p.nbd * p.nbh * p.nbw;
  const int grid = std::min(nbox, device_cus());
  auto kern = b.lbd == 2 ? stem_fwd_ws_kernel<2, 3> : stem_fwd_ws_kernel<3, 2>;
  if (b.lbd == 2 && mode == 1) kern = stem_fwd_ws_kernel<2, 3, 1>;
  if (b.lbd == 2 && mode == 2) kern = stem_fwd_ws_kernel<2, 3, 2>;
  if (b.lbd == 2 && mode == 3) kern = stem_fwd_ws_kernel<2, 3, 3>;
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, kWsLds);
  hipLaunchKernelGGL(kern, dim3(grid), dim3(512), kWsLds, s, p, nbox, nbox, (uint32_t)(p.nvox * 16),
                     (uint32_t)(p.nvox * 128), err);
  return (int)hipGetLastError();
}

int exp_wg(int mode, int ns, const void* x, const void* dy, float* part, int N, int D, int H, int W, hipStream_t s) {
  const int nbox = N * (D / 4) * (H / 4) * (W / 16);
  const int grid = std::min(nbox, device_cus());
  const uint32_t xb = (uint32_t)((long)N * D * H * W * 16), yb = (uint32_t)((long)N * D * H * W * 128);
#define EXPWG(M, NSV)                                                                                           \
  if (mode == M && ns == NSV) {                                                                                 \
    auto k = wg_exp_kernel<4, NSV, M>;                                                                          \
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, NSV * SWGeom<4>::Buf); \
    hipLaunchKernelGGL(k, dim3(grid), dim3(kSWT4), NSV * SWGeom<4>::Buf, s, (const bf16_t*)x, (const bf16_t*)dy,   \
                       part, N, D, H, W, xb, yb);                                                               \
    return (int)hipGetLastError();                                                                              \
  }
  EXPWG(7, 3) EXPWG(6, 3) EXPWG(4, 3) EXPWG(2, 3) EXPWG(0, 3) EXPWG(5, 3) EXPWG(1, 3)
  EXPWG(6, 2) EXPWG(4, 2) EXPWG(7, 2)
#undef EXPWG
  return -1;
}

int exp_stem_fwd_v3(int mode, const void* x, const void* wpack, const float* bias, void* y, float* stats, int N, int D,
                    int H, int W, hipStream_t s) {
  const Box b = fwd_box(D, H, W);
  if (!(b.lbw == 4 && b.lbd + b.lbh == 5 && (b.lbd == 2 || b.lbd == 3))) return -5;
  Conv3Params p;
  p.x0 = x; p.x1 = nullptr; p.c0 = 8; p.c1 = 0;
  p.w = wpack; p.bias = bias; p.y0 = y; p.y1 = nullptr; p.cy0 = 64;
  p.yacc = nullptr; p.stats = stats; p.accumulate = 0;
  p.N = N; p.D = D; p.H = H; p.W = W; p.Cin = 8; p.Cout = 64;
  p.nvox = (long)N * D * H * W;
  p.nchunk = 1; p.chunks_per_split = 1;
  p.lbd = b.lbd; p.lbh = b.lbh; p.lbw = b.lbw;
  p.nbd = cdiv(D, 1 << b.lbd); p.nbh = cdiv(H, 1 << b.lbh); p.nbw = cdiv(W, 1 << b.lbw);
  const int nbox = N * p.nbd * p.nbh * p.nbw;
  const int grid = std::min(nbox, device_cus());
  auto kern = b.lbd == 2 ? stem_fwd_v3_kernel<2, 3> : stem_fwd_v3_kernel<3, 2>;
  if (b.lbd == 2) {
    if (mode == 1) kern = stem_fwd_v3_kernel<2, 3, 1>;
    if (mode == 2) kern = stem_fwd_v3_kernel<2, 3, 2>;
    if (mode == 4) kern = stem_fwd_v3_kernel<2, 3, 4>;
    if (mode == 6) kern = stem_fwd_v3_kernel<2, 3, 6>;
    if (mode == 3) kern = stem_fwd_v3_kernel<2, 3, 3>;
    if (mode == 14) kern = stem_fwd_v3_kernel<2, 3, 14>;
    if (mode == 30) kern = stem_fwd_v3_kernel<2, 3, 30>;
    if (mode == 46) kern = stem_fwd_v3_kernel<2, 3, 46>;
    if (mode == 62) kern = stem_fwd_v3_kernel<2, 3, 62>;
    if (mode == 38) kern = stem_fwd_v3_kernel<2, 3, 38>;
  }
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, kS3Lds);
  hipLaunchKernelGGL(kern, dim3(grid), dim3(512), kS3Lds, s, p, nbox, nbox, (uint32_t)(p.nvox * 16),
                     (uint32_t)(p.nvox * 128));
  return (int)hipGetLastError();
}

int exp_stem_wgrad_v2(const void* x, const void* dy, float* dw, float* ws, int cin_w, int N, int D, int H, int W,
                      hipStream_t s) {
  const int nbox = N * (D / kSWBD) * (H / 4) * (W / 16);
  const int grid = std::min(nbox, device_cus());
  const long xbytes = (long)N * D * H * W * 16, dybytes = (long)N * D * H * W * 128;
  auto kern = stem_wgrad_v2_kernel<kSWBD, kSWNS>;
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, kW2Lds);
  hipLaunchKernelGGL(kern, dim3(grid), dim3(kSWT4), kW2Lds, s, (const bf16_t*)x, (const bf16_t*)dy, ws, N, D, H, W,
                     cin_w, (uint32_t)xbytes, (uint32_t)dybytes);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  const int total = 64 * cin_w * 27;
  hipLaunchKernelGGL(stem_wgrad_reduce_kernel, dim3(cdiv(total, 32)), dim3(256), 0, s, (const float*)ws, grid, total,
                     dw);
  return (int)hipGetLastError();
}

int exp_read_stream(const void* y, long bytes, int grid, float* out, hipStream_t s) {
  hipLaunchKernelGGL(read_stream_kernel, dim3(grid), dim3(512), 0, s, (const u32x4_t*)y, bytes / 16, out);
  return (int)hipGetLastError();
}

}  // extern "C"
