// 3x3x3 / stride 1 / pad 1 convolution for the U-Net DoubleConv blocks, NDHWC, gfx950.
//
// Replaces nn.Conv3d(k=3, padding=1) of models/unet3d.py:29,35 (forward, and the two
// autograd backward products of aten::convolution_backward).
//
//   conv3_fwd   implicit GEMM  Y[v, co] = sum_{tap, ci} X[v + tap, ci] * W[co, ci, tap]
//               M = voxels (a spatial box of <= 512 voxels per workgroup), N = 64 output
//               channels per workgroup, K = 27 * Cin walked as (ci-chunk, tap).  The
//               chunk's (box + halo) input tile is staged once in LDS and re-read for all
//               27 taps through an LDS row offset; weights stream from L2 into registers.
//               Epilogue: + bias, store, per-workgroup BatchNorm partial sums (sum, sumsq).
//               Also serves dgrad (dX = conv(dY, W flipped + transposed)), with
//               `accumulate` and a two-pointer output for the concat split of Up3D.
//   conv3_wgrad dW[tap, co, ci] += sum_v dY[v, co] * X[v + tap, ci]   (K = voxels)
//               Both MFMA operands need the voxel index contiguous: they are read from
//               natural NDHWC LDS tiles with ds_read_b64_tr_b16 (hardware transpose).
//
// bf16 path: v_mfma_f32_32x32x16_bf16; fp32 path (parity build): v_mfma_f32_32x32x2_f32.
#include "common.h"
#include "pcms_hip.h"
#include <algorithm>
#include <cstdlib>
#include <type_traits>
#include <utility>

#include "conv_common.h"

namespace {

// LBD/LBH/LBW >= 0: compile-time box geometry (the hot (4, 8, 16) box: halo decode and tap
// offsets become constant arithmetic); -1: runtime geometry from p.
// MTW: M-tiles per wave (4: 512-voxel boxes; 2: boxes of <= 256 voxels -- level 4's 8x8x4 --
// on all four waves instead of two)
// ablation builds of the general forward / dgrad (0 in the product): bit 1 the fp32 (split)
// chunks after a workgroup's first are not staged, 2 no MFMA phase for them
#ifndef CONV_ABL
#define CONV_ABL 0
#endif
template <typename T, int MINW, int LBD, int LBH, int LBW, int MTW = 4>
__global__ void __launch_bounds__(kThreads, MINW) conv3_fwd_kernel(Conv3Params p) {
  const int lbd_ = LBW >= 0 ? LBD : p.lbd, lbh_ = LBW >= 0 ? LBH : p.lbh, lbw_ = LBW >= 0 ? LBW : p.lbw;
  typedef Traits<T> Tr;
  typedef typename Tr::Frag Frag;
  __shared__ __attribute__((aligned(16))) char lds[kHaloMax * kRowBytes];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r_lane = lane & 31, hsel = lane >> 5;
  // 1-D grid of (box, co block, split), co block fastest in the logical id; the logical id is
  // XCD-aware (dispatch is round-robin over the 8 XCDs): an XCD runs consecutive logical ids,
  // i.e. every co block of a few adjacent boxes, which share their halos in its L2.  (The
  // other order -- an XCD holding every box of a few weight slices -- measured slower at
  // levels 2-3 in round 4: DESIGN.md §0c item 3(b).)
  const int nbox = p.N * p.nbd * p.nbh * p.nbw, nco = p.Cout >> 6;
  const int G = gridDim.x;
  const int lg = (G & 7) == 0 ? (blockIdx.x & 7) * (G >> 3) + (blockIdx.x >> 3) : blockIdx.x;
  const int bx = (lg / nco) % nbox, by = lg % nco;
  const int bz = lg / (nbox * nco);
  int mb = bx;
  const int bwi = mb % p.nbw; mb /= p.nbw;
  const int bhi = mb % p.nbh; mb /= p.nbh;
  const int bdi = mb % p.nbd;
  const int n = mb / p.nbd;
  const int co_base = by * 64;
  const int cbeg = bz * p.chunks_per_split;
  const int cend = min(p.nchunk, cbeg + p.chunks_per_split);
  const int bd = 1 << lbd_, bh = 1 << lbh_, bw = 1 << lbw_;
  const int boxvol = bd * bh * bw;
  const int d0 = bdi * bd, h0 = bhi * bh, w0 = bwi * bw;
  const int HH = bh + 2, HW = bw + 2;
  const int HV = (bd + 2) * HH * HW;

  const bool w16 = lbw_ == 4;
  const int prow = w16 ? perm32(r_lane) : r_lane;
  int hb[MTW];
#pragma unroll
  for (int mt = 0; mt < MTW; ++mt) {
    int r = wave * (32 * MTW) + mt * 32 + prow;
    if (r >= boxvol) r = 0;
    int rd = r >> (lbh_ + lbw_), rh = (r >> lbw_) & (bh - 1), rw = r & (bw - 1);
    hb[mt] = (rd * HH + rh) * HW + rw;
  }
  const bool wave_active = wave * (32 * MTW) < boxvol;

  // fp32 data (x3_t / x6_t): the fp32 halo split into bf16 parts in LDS, three MFMAs per
  // (M-tile, N-tile, tap) instead of two
  constexpr bool kX3 = std::is_same<T, x3_t>::value, kX6 = std::is_same<T, x6_t>::value;
  constexpr bool kSplit = kX3 || kX6;
  typedef typename Tr::Mem M;
  f32x16_t acc[MTW][2];
#pragma unroll
  for (int i = 0; i < MTW; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  const M* x0 = (const M*)p.x0;
  const M* x1 = (const M*)p.x1;
  const bf16_t* wp = (const bf16_t*)p.w;
  const long plane = (long)p.H * p.W;

  for (int chunk = cbeg; chunk < cend; ++chunk) {
#if CONV_ABL & 1  // ablation builds only (wrong results, timing): fp32 chunks after the first not staged
    if (kSplit && chunk > cbeg) goto compute_chunk;
#endif
    __syncthreads();
    // ---- stage the halo tile of this chunk by LDS-DMA: piece p (16 B) -> LDS [16p, 16p+16).
    // The LDS image is lane-linear, so the slot swizzle is applied to the SOURCE address
    // (physical slot qp of row hv holds logical slot qp ^ swz(hv)); out-of-range pieces
    // read the zero page.  All pieces are in flight at once (no register staging).
    for (int base = wave * 64; base < HV * 4; base += kThreads) {
      const int pc = base + lane;
      const int hv = pc >> 2;
      const int ql = (pc & 3) ^ swz(hv);
      const void* src = g_zero16;
      if (pc < HV * 4) {
        const int hw_ = hv % HW, t_ = hv / HW, hh_ = t_ % HH, hd_ = t_ / HH;
        const int gd = d0 + hd_ - 1, gh = h0 + hh_ - 1, gw = w0 + hw_ - 1;
        const int c = chunk * Tr::CK + ql * Tr::VEC;
        if (gd >= 0 && gd < p.D && gh >= 0 && gh < p.H && gw >= 0 && gw < p.W && c < p.Cin &&
            ql * Tr::VEC < Tr::CK) {  // (x6: the row's slots 2, 3 stay zero)
          const long vox = ((long)n * p.D + gd) * plane + (long)gh * p.W + gw;
          src = (c < p.c0) ? (const void*)(x0 + vox * p.c0 + c) : (const void*)(x1 + vox * p.c1 + (c - p.c0));
        }
      }
      __builtin_amdgcn_global_load_lds(src, (LDS_AS void*)(lds + base * 16), 16, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if constexpr (kX6) {
      // split every 8-channel fp32 row in place into logical slots [h | m | l | 0]
      for (int r = tid; r < HV; r += kThreads) {
        char* row = lds + r * kRowBytes;
        const int sw = swz(r);
        const f32x4_t q0 = *reinterpret_cast<const f32x4_t*>(row + ((0 ^ sw) * 16));
        const f32x4_t q1 = *reinterpret_cast<const f32x4_t*>(row + ((1 ^ sw) * 16));
        const float f[8] = {q0[0], q0[1], q0[2], q0[3], q1[0], q1[1], q1[2], q1[3]};
        u32x4_t h, m, l;
        split3x8(f, h, m, l);
        *reinterpret_cast<u32x4_t*>(row + ((0 ^ sw) * 16)) = h;
        *reinterpret_cast<u32x4_t*>(row + ((1 ^ sw) * 16)) = m;
        *reinterpret_cast<u32x4_t*>(row + ((2 ^ sw) * 16)) = l;
      }
      __syncthreads();
    }
    if constexpr (kX3) {
      // split every 16-channel fp32 row in place: logical 16-B slot s of the row (physical
      // s ^ swz) = [hi 0-7, hi 8-15, lo 0-7, lo 8-15], so lds_a(ks = 0 / 1) reads hi / lo
      for (int r = tid; r < HV; r += kThreads) {
        char* row = lds + r * kRowBytes;
        const int sw = swz(r);
        f32x4_t q[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) q[k] = *reinterpret_cast<const f32x4_t*>(row + ((k ^ sw) * 16));
        u32x4_t o[4];
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            const u32x2_t hl = split2(q[k][2 * i], q[k][2 * i + 1]);
            o[k >> 1][(k & 1) * 2 + i] = hl[0];
            o[2 + (k >> 1)][(k & 1) * 2 + i] = hl[1];
          }
#pragma unroll
        for (int s = 0; s < 4; ++s) *reinterpret_cast<u32x4_t*>(row + ((s ^ sw) * 16)) = o[s];
      }
      __syncthreads();
    }
#if CONV_ABL & 1
  compute_chunk:
#endif
    if (!wave_active) continue;
#if CONV_ABL & 2  // ablation builds only: no MFMA phase for the fp32 data
    if (kSplit) continue;
#endif

    const bf16_t* wchunk = wp + (long)chunk * 27 * p.Cout * Tr::WK;
    Frag bset[2][2][Tr::KS];
    auto load_b = [&](Frag (&dst)[2][Tr::KS], int tap) {
      if constexpr (std::is_same<T, bf16_t>::value) {
        // fragment-major pack (pack_bf16_off): block (row tile, ks) = one contiguous 1 KiB
        const bf16_t* wt = wchunk + ((long)tap * p.Cout + co_base) * 32 + lane * 8;
#pragma unroll
        for (int nt = 0; nt < 2; ++nt)
#pragma unroll
          for (int ks = 0; ks < Tr::KS; ++ks)
            dst[nt][ks] = *reinterpret_cast<const s16x8_t*>(wt + nt * 1024 + ks * 512);
      } else {
        const bf16_t* wt = wchunk + ((long)tap * p.Cout + co_base + r_lane) * Tr::WK;
#pragma unroll
        for (int nt = 0; nt < 2; ++nt)
#pragma unroll
          for (int ks = 0; ks < Tr::KS; ++ks) dst[nt][ks] = gl_b(wt + nt * 32 * Tr::WK, ks, hsel);
      }
    };
    load_b(bset[0], 0);
    // The A fragments roll through one register set: right after M-tile mt's MFMAs of tap t
    // its fragment of tap t + 1 is read (15 MFMAs of slack before its first use) instead of
    // one read -> wait -> two MFMAs per fragment.  B: two register sets, tap t + 1 loaded
    // while tap t computes (a third set, two taps ahead, pushed the kernel past 256 VGPRs into
    // spills with a reload inside this loop); taps walked two (kd, kh) rows per trip so every
    // set index is a compile-time constant.
    // x6: a[0] = [h|m], a[1] = [h|l] (logical slot 2 * hsel)
    auto frag1 = [&](int row) __attribute__((always_inline)) {
      if constexpr (kX6) return lds_slot(lds, row, 2 * hsel);
      else return lds_a(lds, row, 1, hsel);
    };
    s16x8_t a[2][MTW];
#pragma unroll
    for (int mt = 0; mt < MTW; ++mt) {
      a[0][mt] = lds_a(lds, hb[mt], 0, hsel);
      a[1][mt] = frag1(hb[mt]);
    }
    auto tap_step = [&](int tap, int set, const int (&hbk)[MTW]) {
      load_b(bset[set ^ 1], min(tap + 1, 26));
      __builtin_amdgcn_sched_barrier(0);  // keep the prefetch ahead of this tap's MFMAs
      const int tn = tap + 1 < 27 ? tap + 1 : 0;
      const int offn = ((tn / 9) * HH + (tn / 3) % 3) * HW + tn % 3;
      if constexpr (kSplit) {
        // x3: hi*hi + lo*hi + hi*lo (a[0] = hi, a[1] = lo; B ks 0 = hi, 1 = lo)
        // x6: [h|m].[h|h] + [h|l].[m|h] + [h|m].[l|m] (a[0], a[1]; B ks 0, 1, 2)
        constexpr int b1 = kX6 ? 1 : 0, b2 = kX6 ? 2 : 1;
#pragma unroll
        for (int mt = 0; mt < MTW; ++mt) {
#pragma unroll
          for (int nt = 0; nt < 2; ++nt) acc[mt][nt] = mfma(a[0][mt], bset[set][nt][0], acc[mt][nt]);
#pragma unroll
          for (int nt = 0; nt < 2; ++nt) acc[mt][nt] = mfma(a[1][mt], bset[set][nt][b1], acc[mt][nt]);
          a[1][mt] = frag1(hbk[mt] + offn);
#pragma unroll
          for (int nt = 0; nt < 2; ++nt) acc[mt][nt] = mfma(a[0][mt], bset[set][nt][b2], acc[mt][nt]);
          a[0][mt] = lds_a(lds, hbk[mt] + offn, 0, hsel);
        }
#pragma unroll
        for (int i = 0; i < 2 * MTW; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, 3, 0);  // 3 MFMA
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // 1 DS read
        }
      } else {
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
          for (int mt = 0; mt < MTW; ++mt) {
#pragma unroll
            for (int nt = 0; nt < 2; ++nt) acc[mt][nt] = mfma(a[ks][mt], bset[set][nt][ks], acc[mt][nt]);
            a[ks][mt] = lds_a(lds, hbk[mt] + offn, ks, hsel);
          }
        // (the scheduler would otherwise sink all eight reads below the last MFMA)
#pragma unroll
        for (int i = 0; i < 2 * MTW; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);  // 2 MFMA
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // 1 DS read
        }
      }
    };
    for (int kdh = 0; kdh < 8; kdh += 2) {
      // row bases from an opaque copy: the fragment addresses are recomputed per trip rather
      // than hoisted out of the loops (and spilled)
      int hbk[MTW];
#pragma unroll
      for (int mt = 0; mt < MTW; ++mt) hbk[mt] = opaque(hb[mt]);
#pragma unroll
      for (int j = 0; j < 6; ++j) tap_step(kdh * 3 + j, j & 1, hbk);
    }
    {
      int hbk[MTW];
#pragma unroll
      for (int mt = 0; mt < MTW; ++mt) hbk[mt] = opaque(hb[mt]);
#pragma unroll
      for (int j = 0; j < 3; ++j) tap_step(24 + j, j & 1, hbk);
    }
  }

  // ---- epilogue ----
  // BatchNorm partials per workgroup row: (sum, M2 = sum of squared deviations from the
  // row's own mean) + the row's voxel count.  Each wave first forms its own per-channel
  // mean (two passes over the accumulator registers), waves are merged with Chan's formula:
  // no E[x^2] - E[x]^2 cancellation (BN over few voxels / large |mean| / std).
  float s1[2] = {0.f, 0.f}, s2[2] = {0.f, 0.f};
  float bias_l[2] = {0.f, 0.f};
  if (p.bias) {
    bias_l[0] = p.bias[co_base + r_lane];
    bias_l[1] = p.bias[co_base + 32 + r_lane];
  }
  const bool want_stats = p.stats && !p.yacc;
  const bool interior = d0 + bd <= p.D && h0 + bh <= p.H && w0 + bw <= p.W;
  uint64_t vmask = 0;  // bit mt * 16 + e: row valid
  if (wave_active) {
#pragma unroll
    for (int mt = 0; mt < MTW; ++mt)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int rr = (e & 3) + 8 * (e >> 2) + 4 * hsel;
        const int r = wave * (32 * MTW) + mt * 32 + (w16 ? perm32(rr) : rr);
        bool valid = r < boxvol;
        if (valid && !interior) {
          const int rd = r >> (lbh_ + lbw_), rh = (r >> lbw_) & (bh - 1), rw = r & (bw - 1);
          valid = d0 + rd < p.D && h0 + rh < p.H && w0 + rw < p.W;
        }
        if (valid) vmask |= 1ull << (mt * 16 + e);
      }
  }
  constexpr int kRedOff = 512 * 64 * 2;  // bf16 C tile [512][64] occupies the first 64 KiB
  // (PCMS_CONV_RELU, eval with the BatchNorm folded into w / b: tested where used, from the
  // kernel argument -- a flag held across the epilogue cost a spill)
  if (!kSplit && !p.yacc && !(p.accumulate & PCMS_CONV_ACCUMULATE)) {
    // bf16 fast path: + bias, stats from the fp32 values, C tile -> LDS (box order), then
    // 16-byte coalesced stores (one box row = a contiguous w-run of voxels).
    __syncthreads();  // every wave is done reading the halo
    bf16_t* ct = reinterpret_cast<bf16_t*>(lds);
    if (wave_active) {
#pragma unroll
      for (int mt = 0; mt < MTW; ++mt) {
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int rr = (e & 3) + 8 * (e >> 2) + 4 * hsel;
          const int r = wave * (32 * MTW) + mt * 32 + (w16 ? perm32(rr) : rr);
          const bool valid = (vmask >> (mt * 16 + e)) & 1;
#pragma unroll
          for (int nt = 0; nt < 2; ++nt) {
            const float v = acc[mt][nt][e] + bias_l[nt];
            ct[r * 64 + nt * 32 + r_lane] = f2bf(v);
            if (valid) s1[nt] += v;
          }
        }
      }
    }
    __syncthreads();
    for (int pc = tid; pc < boxvol * 8; pc += kThreads) {
      const int r = pc >> 3, q = pc & 7;
      const int rd = r >> (lbh_ + lbw_), rh = (r >> lbw_) & (bh - 1), rw = r & (bw - 1);
      const int gd = d0 + rd, gh = h0 + rh, gw = w0 + rw;
      if (!interior && (gd >= p.D || gh >= p.H || gw >= p.W)) continue;
      const long vox = ((long)n * p.D + gd) * plane + (long)gh * p.W + gw;
      const int co = co_base + q * 8;
      M* dst = (co < p.cy0) ? (M*)p.y0 + vox * p.cy0 + co : (M*)p.y1 + vox * (p.Cout - p.cy0) + (co - p.cy0);
      u32x4_t o = *reinterpret_cast<const u32x4_t*>(ct + r * 64 + q * 8);
      if (p.accumulate & PCMS_CONV_RELU) o = relu_bf16x8(o);
      *reinterpret_cast<u32x4_t*>(dst) = o;
    }
  } else if (wave_active) {
#pragma unroll
    for (int mt = 0; mt < MTW; ++mt) {
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        if (!((vmask >> (mt * 16 + e)) & 1)) continue;
        const int rr = (e & 3) + 8 * (e >> 2) + 4 * hsel;
        const int r = wave * (32 * MTW) + mt * 32 + (w16 ? perm32(rr) : rr);
        const int rd = r >> (lbh_ + lbw_), rh = (r >> lbw_) & (bh - 1), rw = r & (bw - 1);
        const int gd = d0 + rd, gh = h0 + rh, gw = w0 + rw;
        const long vox = ((long)n * p.D + gd) * plane + (long)gh * p.W + gw;
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
          const int co = co_base + nt * 32 + r_lane;
          float v = acc[mt][nt][e];
          if (p.yacc) {  // split-K: this split's own fp32 slab (summed in a fixed order later)
            p.yacc[((long)bz * p.nvox + vox) * p.Cout + co] = v;
            continue;
          }
          v += bias_l[nt];
          M* dst = (co < p.cy0) ? (M*)p.y0 + vox * p.cy0 + co
                                : (M*)p.y1 + vox * (p.Cout - p.cy0) + (co - p.cy0);
          if (p.accumulate & PCMS_CONV_ACCUMULATE) v += Elem<M>::ld(dst);  // (stats are refused with accumulate)
          if (p.accumulate & PCMS_CONV_RELU) v = fmaxf(v, 0.f);
          Elem<M>::st(dst, v);
          s1[nt] += v;
        }
      }
    }
  }
  if (want_stats) {
    // wave-level mean per channel (rows of a channel live in lanes r_lane and r_lane + 32)
    const float nw = (float)(__popcll(vmask) + __shfl_xor(__popcll(vmask), 32, 64));
    float mw[2];
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      s1[nt] += __shfl_xor(s1[nt], 32, 64);
      mw[nt] = nw > 0.f ? s1[nt] / nw : 0.f;
    }
    // squared deviations about the rounded wave mean, corrected by (sum d)^2 / n
    float sd[2] = {0.f, 0.f};
    if (wave_active) {
#pragma unroll
      for (int mt = 0; mt < MTW; ++mt)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          if (!((vmask >> (mt * 16 + e)) & 1)) continue;
#pragma unroll
          for (int nt = 0; nt < 2; ++nt) {
            const float d = acc[mt][nt][e] + bias_l[nt] - mw[nt];
            s2[nt] += d * d;
            sd[nt] += d;
          }
        }
    }
    __syncthreads();  // halo / C tile no longer read: reuse LDS for the cross-wave reduction
    float* red = reinterpret_cast<float*>(lds + (kSplit ? 0 : kRedOff));
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      s2[nt] += __shfl_xor(s2[nt], 32, 64);
      sd[nt] += __shfl_xor(sd[nt], 32, 64);
      if (nw > 0.f) s2[nt] -= sd[nt] * sd[nt] / nw;
      if (hsel == 0) {
        float* rp = red + (wave * 64 + nt * 32 + r_lane) * 3;
        rp[0] = s1[nt];
        rp[1] = s2[nt];
        rp[2] = nw;
      }
    }
    __syncthreads();
    if (tid < 64) {
      float S = 0.f, Nn = 0.f;
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        S += red[(w * 64 + tid) * 3 + 0];
        Nn += red[(w * 64 + tid) * 3 + 2];
      }
      const float m = Nn > 0.f ? S / Nn : 0.f;
      float M2 = 0.f, sdd = 0.f;
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        const float c = red[(w * 64 + tid) * 3 + 2];
        if (c > 0.f) {
          const float d = red[(w * 64 + tid) * 3 + 0] / c - m;
          M2 += red[(w * 64 + tid) * 3 + 1] + c * d * d;
          sdd += c * d;
        }
      }
      if (Nn > 0.f) M2 -= sdd * sdd / Nn;
      float* st = p.stats + ((long)bx * p.Cout + co_base + tid) * 2;
      st[0] = S;
      st[1] = M2;
      if (tid == 0 && by == 0) p.stats[(long)nbox * p.Cout * 2 + bx] = Nn;
    }
  }
}

// ------------------------------------------------------------------------------------
// weight-gradient kernel
// ------------------------------------------------------------------------------------
__device__ __forceinline__ f32x4_t mfma16(s16x8_t a, s16x8_t b, f32x4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b), c,
                                                 0, 0, 0);
}

constexpr int kWThreads = 512;          // 8 waves: wave = (co-tile, tap-group)
// ablation builds only (tests/tools/wgrad_abl.py; 0 in the product): bit 1 the direct flush's
// global stores dropped, 2 no staging after a workgroup's first box, 4 no MFMA phase, 8 no
// wait for the next box's DMA at a box's end, 16 the spread pieces' addresses computed but
// read nothing (zeros land in LDS), 32 the spread pieces read fixed in-range addresses (no
// address arithmetic) -- wrong results: timing only
#ifndef WGRAD_ABL
#define WGRAD_ABL 0
#endif
// A/B builds: bit 0 s_setprio 1 for waves 4-7 of the weight gradient, bit 1 of the 8-deep
// 16x16x32 conv (MI355X_MICROARCH.md, two waves per SIMD item 4); 0 in the product
#ifndef PCMS_SETPRIO
#define PCMS_SETPRIO 0
#endif
constexpr int kWHaloMax = 720;          // halo rows (box <= 256 voxels)

template <typename T> struct WTraits;
template <> struct WTraits<bf16_t> {
  static constexpr int BV = 256;        // voxels per staged box
  static constexpr int KV = 16;         // voxels per MFMA
  static constexpr int NBUF = 2;
  static constexpr int DYROW = 128;     // 64 co x 2 B
  static constexpr int XROW = 64;       // 32 ci x 2 B
  static constexpr int VEC = 8;
  static constexpr int HALO = kWHaloMax;
  static constexpr int NPART = 1;
  typedef s16x8_t Frag;
};
template <> struct WTraits<x6_t> {
  // boxes of <= 64 voxels (round 6): the h, m, l tiles (3 x 24 KB) plus the fp32 LDS-DMA
  // target of the NEXT box (48 KB) fit in LDS, so the box stream no longer stops the MFMAs
  static constexpr int BV = 64;         // voxels per staged box
  static constexpr int KV = 8;          // voxels per MFMA k-step (K halves concatenated)
  static constexpr int NBUF = 1;
  static constexpr int DYROW = 128;
  static constexpr int XROW = 64;
  static constexpr int VEC = 4;
  static constexpr int HALO = 256;
  static constexpr int NPART = 3;
  // the fp32 box as it arrives by LDS-DMA: dy [BV][64 co] then the x halo [HALO][32 ci] (+ one
  // wave-instruction of slack: a halo's last DMA may run past its rows, reading zeros)
  static constexpr int RAWDY = BV * 64 * 4;
  static constexpr int RAWBYTES = RAWDY + (HALO * 8 + 64) * 16;
  typedef s16x8_t Frag;
};
template <> struct WTraits<x3_t> {
  static constexpr int BV = 128;        // voxels per staged box (hi + lo tiles: 2 x 62 KB)
  static constexpr int KV = 16;
  static constexpr int NBUF = 1;
  static constexpr int DYROW = 128;     // LDS rows as bf16 (one tile per half)
  static constexpr int XROW = 64;
  static constexpr int VEC = 4;         // fp32 elements per 16-B global piece
  static constexpr int HALO = kWHaloMax;
  static constexpr int NPART = 2;
  typedef s16x8_t Frag;
};

struct WgradParams {
  const void* x0; const void* x1; int c0; int c1;
  const void* dy;
  float* dwt;            // fp32 workspace: one [27][Cout][Cin] partial row per split
  int N, D, H, W, Cin, Cout;
  int lbd, lbh, lbw, nbd, nbh, nbw;
  int nbox, boxes_per_split;
  int nco, nci;          // 64-channel output blocks, 32-channel input blocks
  int dma;               // bf16: stage by buffer LDS-DMA (byte sizes below < 2^31)
  uint32_t x0bytes, x1bytes, dybytes;
  float* dw;             // direct (one split, bf16): dw [Cout][cw][27] += through an LDS transpose
  int cw, direct;
  int store;             // PCMS_GRAD_STORE: dw = (the first writer of a fresh gradient), not +=
  int ntg;               // tap groups (TG kernels: 2, taps [0, 16) / [16, 27) per workgroup)
  // BNIN kernels (pcms_conv3_wgrad_bnin): x is relu(x0 * isc + ish) per input channel
  const float* isc = nullptr; const float* ish = nullptr;
};


// TG: the taps are split over two workgroups per (tile, split) -- for grids of few boxes,
// where splitting the voxels instead would add partial rows and a reduction pass
// BNIN (bf16, LDS-DMA staging, one source): the staged x halo is relu(x * isc + ish), applied
// in LDS by the thread that staged each piece, after its DMA landed and before the barrier that
// publishes the buffer (the BatchNorm + ReLU of the layer below, fused as in
// conv3_fwd_big_kernel<true>); out-of-range pieces (zero padding) stay zero
// K16 (bf16, compile-time box, no TG): v_mfma_f32_16x16x32_bf16 instead of 32x32x16 -- the same
// LDS reads per FLOP (K = 32 voxels per step: 8 A + 4 B transposed reads per tap pair of
// ci tiles), the MFMA shape that runs the power-capped big-box convs at a higher clock
// (profiles/r5_mfma_shape_probe.txt).  acc16[j][ct][t]: tap j, 16-co tile ct, 16-ci tile t.
template <typename T, int LBD, int LBH, int LBW, bool TG = false, bool P4 = false, bool BNIN = false,
          bool K16 = false>
__global__ void __launch_bounds__(kWThreads, 1) conv3_wgrad_kernel(WgradParams p) {
  static_assert(!K16 || (std::is_same<T, bf16_t>::value && LBW >= 2 && !TG), "K16: bf16 fixed boxes");
  const int lbd_ = LBW >= 0 ? LBD : p.lbd, lbh_ = LBW >= 0 ? LBH : p.lbh, lbw_ = LBW >= 0 ? LBW : p.lbw;
  typedef WTraits<T> Tr;
  typedef typename Tr::Frag Frag;
  constexpr int DYBYTES = Tr::BV * Tr::DYROW;
  constexpr int XBYTES = Tr::HALO * Tr::XROW;
  constexpr int BUFBYTES = DYBYTES + XBYTES;
  extern __shared__ __attribute__((aligned(16))) char wlds[];

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hsel = lane >> 5;
#if PCMS_SETPRIO & 1
  // static priority for the second-dispatched half (waves 4-7: each SIMD's younger wave)
  if (wave >= 4) __builtin_amdgcn_s_setprio(1);
#endif
  // wave w owns taps w, w + 8, w + 16 (, w + 24) for BOTH co tiles, so each B (x) fragment
  // feeds 2 MFMAs: 1.5 LDS reads per MFMA instead of 2.3 (8 accumulators)
  // fp32 data, split-bf16 products: x3 (hi, lo tiles) / x6 (h, m, l tiles), the parts
  // BUFBYTES apart
  constexpr bool kX3 = std::is_same<T, x3_t>::value, kX6 = std::is_same<T, x6_t>::value;
  typedef typename std::conditional<kX3 || kX6, float, bf16_t>::type M;
  // 1-D grid, logical id XCD-aware (dispatch is round-robin over 8 XCDs: consecutive logical
  // ids land on one XCD at about the same time), tile (co block, ci block) fastest: the
  // workgroups of one split that share its dy boxes (and its halos) share an L2
  const int G = gridDim.x, ntile = p.nco * p.nci;
  const int lg = (G & 7) == 0 ? (blockIdx.x & 7) * (G >> 3) + (blockIdx.x >> 3) : blockIdx.x;
  const int tile = lg % ntile, split = lg / ntile / (TG ? 2 : 1);
  // the wave's taps: main taps tb + 8 j (j < NJ, accumulators j and 4 + j) and, where it
  // exists, one more at tb + 8 NJ (accumulators 3 and 7).  TG group 0: taps w, w + 8;
  // group 1: 16 + w, 24 + w (waves 0-2)
  const int tgrp = TG ? (lg / ntile) & 1 : 0;
  constexpr int NJ = TG ? 1 : 3;
  const int tb = 16 * tgrp + wave;
  const bool four = TG ? (tgrp == 0 || wave < 3) : wave < 3;
  auto owned = [&](int j) __attribute__((always_inline)) { return j < NJ || (j == 3 && four); };
  auto tapof = [&](int j) __attribute__((always_inline)) { return tb + 8 * (j < NJ ? j : NJ); };
  const int co_base = (tile % p.nco) * 64;
  const int ci_base = (tile / p.nco) * 32;
  // fp32 build, <= 8 input channels (the stem): the 32 MFMA columns hold 4 taps x 8 channels
  // (column n = tap 4 wave + n / 8, channel n % 8; waves 0-6 own the 7 tap groups) instead of
  // one tap x 32 channels of which 24 are padding -- 3.9x fewer MFMAs per box
  constexpr bool pack4 = kX6 && P4;  // the host launches P4 for Cin <= 8 only
  const int bd = 1 << lbd_, bh = 1 << lbh_, bw = 1 << lbw_;
  const int HH = bh + 2, HW = bw + 2;
  const int HV = (bd + 2) * HH * HW;
  const int boxvol = bd * bh * bw;
  const long plane = (long)p.H * p.W;
  const M* x0 = (const M*)p.x0;
  const M* x1 = (const M*)p.x1;
  const M* dy = (const M*)p.dy;

  const int b_beg = split * p.boxes_per_split;
  const int b_end = min(p.nbox, b_beg + p.boxes_per_split);

  f32x16_t acc[8];
#pragma unroll
  for (int t = 0; t < 8; ++t)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[t][e] = 0.f;
  f32x4_t acc16[4][4][2];
  if constexpr (K16) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int t = 0; t < 2; ++t) acc16[j][c][t] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
  }

  // register staging: pieces of 16 B
  constexpr int DYP = Tr::BV * Tr::DYROW / 16;
  const int XP = HV * Tr::XROW / 16;
  constexpr int MAXP = Tr::NBUF == 2 ? (DYP + kWHaloMax * Tr::XROW / 16 + kWThreads - 1) / kWThreads : 1;
  u32x4_t stg[MAXP];

  auto box_origin = [&](int b, int& n, int& d0, int& h0, int& w0) {
    int bwi = b % p.nbw; b /= p.nbw;
    int bhi = b % p.nbh; b /= p.nbh;
    int bdi = b % p.nbd;
    n = b / p.nbd;
    d0 = bdi * bd; h0 = bhi * bh; w0 = bwi * bw;
  };
  auto stage_load = [&](int b) {
    int n, d0, h0, w0;
    box_origin(b, n, d0, h0, w0);
#pragma unroll
    for (int i = 0; i < MAXP; ++i) {
      // one unconditional 16-B load per piece (invalid pieces read the zero page): a
      // conditional load merged with a zero default makes the compiler drain vmcnt before
      // the merge, serialising the prefetch with the compute it should overlap
      const int pc = tid + i * kWThreads;
      const void* src = g_zero16;
      if (pc < DYP) {
        const int r = pc / (Tr::DYROW / 16), q = pc % (Tr::DYROW / 16);
        if (r < boxvol) {
          const int rd = r >> (lbh_ + lbw_), rh = (r >> lbw_) & (bh - 1), rw = r & (bw - 1);
          const int gd = d0 + rd, gh = h0 + rh, gw = w0 + rw;
          if (gd < p.D && gh < p.H && gw < p.W) {
            const long vox = ((long)n * p.D + gd) * plane + (long)gh * p.W + gw;
            src = dy + vox * p.Cout + co_base + q * Tr::VEC;
          }
        }
      } else if (pc < DYP + XP) {
        const int hp = pc - DYP;
        const int hv = hp / (Tr::XROW / 16), q = hp % (Tr::XROW / 16);
        const int hw_ = hv % HW, t_ = hv / HW, hh_ = t_ % HH, hd_ = t_ / HH;
        const int gd = d0 + hd_ - 1, gh = h0 + hh_ - 1, gw = w0 + hw_ - 1;
        const int c = ci_base + q * Tr::VEC;
        if (gd >= 0 && gd < p.D && gh >= 0 && gh < p.H && gw >= 0 && gw < p.W && c < p.Cin) {
          const long vox = ((long)n * p.D + gd) * plane + (long)gh * p.W + gw;
          src = (c < p.c0) ? (const void*)(x0 + vox * p.c0 + c) : (const void*)(x1 + vox * p.c1 + (c - p.c0));
        }
      }
      stg[i] = *reinterpret_cast<const u32x4_t*>(src);
    }
  };
  auto stage_store = [&](char* buf) {
#pragma unroll
    for (int i = 0; i < MAXP; ++i) {
      const int pc = tid + i * kWThreads;
      if (pc < DYP) {
        const int r = pc / (Tr::DYROW / 16), q = pc % (Tr::DYROW / 16);
        int off;
        if (sizeof(T) == 2) off = dy_off_bf16(r, q * 8);
        else off = r * Tr::DYROW + q * 16;
        *reinterpret_cast<u32x4_t*>(buf + off) = stg[i];
      } else if (pc < DYP + XP) {
        const int hp = pc - DYP;
        *reinterpret_cast<u32x4_t*>(buf + DYBYTES + hp * 16) = stg[i];
      }
    }
  };

  // fp32 build: every 16-B piece (4 fp32) of the box's dy tile and x halo loaded into
  // registers (all in flight), then split into the hi tile at buf and the lo tile at
  // buf + BUFBYTES (the bf16 layouts: dy_off_bf16 rows, 64-B halo rows)
  auto stage_x3 = [&](char* buf, int b) {
    int n, d0, h0, w0;
    box_origin(b, n, d0, h0, w0);
    constexpr int DYQ = Tr::BV * 16;                      // 64 co / 4 per piece
    constexpr int XQMAX = Tr::HALO * 8;                   // 32 ci / 4
    constexpr int PER = (DYQ + XQMAX + kWThreads - 1) / kWThreads;
    constexpr int RND = 8;                                // pieces in flight per thread (VGPRs)
    const int XQ = HV * 8;
#pragma unroll
    for (int i0 = 0; i0 < PER; i0 += RND) {
      f32x4_t v[RND];
#pragma unroll
      for (int i = 0; i < RND; ++i) {
        const int pc = tid + (i0 + i) * kWThreads;
        const float* src = reinterpret_cast<const float*>(g_zero16);
        if (pc < DYQ) {
          const int r = pc >> 4, q = pc & 15;
          const int rd = r >> (lbh_ + lbw_), rh = (r >> lbw_) & (bh - 1), rw = r & (bw - 1);
          const int gd = d0 + rd, gh = h0 + rh, gw = w0 + rw;
          if (r < boxvol && gd < p.D && gh < p.H && gw < p.W)
            src = reinterpret_cast<const float*>(dy) + (((long)n * p.D + gd) * plane + (long)gh * p.W + gw) * p.Cout + co_base + q * 4;
        } else if (pc < DYQ + XQ) {
          const int hp = pc - DYQ, hv = hp >> 3, q = hp & 7;
          const int hw_ = hv % HW, t_ = hv / HW, hh_ = t_ % HH, hd_ = t_ / HH;
          const int gd = d0 + hd_ - 1, gh = h0 + hh_ - 1, gw = w0 + hw_ - 1;
          const int c = ci_base + q * 4;
          if (gd >= 0 && gd < p.D && gh >= 0 && gh < p.H && gw >= 0 && gw < p.W && c < p.Cin) {
            const long vox = ((long)n * p.D + gd) * plane + (long)gh * p.W + gw;
            src = (c < p.c0) ? reinterpret_cast<const float*>(x0) + vox * p.c0 + c
                             : reinterpret_cast<const float*>(x1) + vox * p.c1 + (c - p.c0);
          }
        }
        v[i] = *reinterpret_cast<const f32x4_t*>(src);
      }
#pragma unroll
      for (int i = 0; i < RND; ++i) {
        const int pc = tid + (i0 + i) * kWThreads;
        int off;
        if (pc < DYQ) off = dy_off_bf16(pc >> 4, (pc & 15) * 4);
        else if (pc < DYQ + XQ) off = DYBYTES + (pc - DYQ) * 8;
        else continue;
        if constexpr (kX6) {
          const float f[8] = {v[i][0], v[i][1], v[i][2], v[i][3], 0.f, 0.f, 0.f, 0.f};
          u32x4_t h, m, l;
          split3x8(f, h, m, l);
          *reinterpret_cast<u32x2_t*>(buf + off) = (u32x2_t){h[0], h[1]};
          *reinterpret_cast<u32x2_t*>(buf + BUFBYTES + off) = (u32x2_t){m[0], m[1]};
          *reinterpret_cast<u32x2_t*>(buf + 2 * BUFBYTES + off) = (u32x2_t){l[0], l[1]};
        } else {
          const u32x2_t h01 = split2(v[i][0], v[i][1]), h23 = split2(v[i][2], v[i][3]);
          *reinterpret_cast<u32x2_t*>(buf + off) = (u32x2_t){h01[0], h23[0]};
          *reinterpret_cast<u32x2_t*>(buf + BUFBYTES + off) = (u32x2_t){h01[1], h23[1]};
        }
      }
    }
  };

  // fp32 build with LDS-DMA (p.dma): the box's fp32 dy tile and x halo into the raw buffer
  // after the part tiles (16-B pieces, one wave-instruction of 64 consecutive pieces each;
  // padding / out-of-volume pieces read zeros), and the split of the landed box into the tiles
  auto stage_raw = [&](int b) __attribute__((always_inline)) {
    if constexpr (kX6) {
      int n, d0, h0, w0;
      box_origin(b, n, d0, h0, w0);
      const uint32_t lb0 = lds_addr(wlds + Tr::NPART * BUFBYTES);
      const bool first = ci_base < p.c0;  // a 32-channel block lies in one source
      const i32x4_t xr = buffer_desc(first ? p.x0 : p.x1, first ? p.x0bytes : p.x1bytes);
      const i32x4_t dr = buffer_desc(p.dy, p.dybytes);
      const int xs = first ? p.c0 : p.c1, xc = first ? ci_base : ci_base - p.c0;
      constexpr int DYQ = Tr::BV * 16;  // 16 pieces of 4 fp32 per voxel (64 co)
      constexpr int RP = (DYQ + Tr::HALO * 8 + kWThreads - 1) / kWThreads;
      static_assert(DYQ % 64 == 0, "dy pieces in whole wave-instructions");
      const int XQ = HV * 8;            // 8 pieces per halo voxel (32 ci)
#pragma unroll
      for (int i = 0; i < RP; ++i) {
        const int pc0 = (tid & ~63) + i * kWThreads;  // wave-uniform first piece
        if (pc0 >= DYQ + XQ) break;
        const int pc = pc0 + lane;
        uint32_t voff = kOOB;
        if (pc0 < DYQ) {
          const int r = pc >> 4, q = pc & 15;
          if (r < boxvol) {
            const int rd = r >> (lbh_ + lbw_), rh = (r >> lbw_) & (bh - 1), rw = r & (bw - 1);
            const int gd = d0 + rd, gh = h0 + rh, gw = w0 + rw;
            if (gd < p.D && gh < p.H && gw < p.W)
              voff = (uint32_t)(((((n * p.D + gd) * p.H + gh) * p.W + gw) * p.Cout + co_base + q * 4) * 4);
          }
          dma16(dr, __builtin_amdgcn_readfirstlane(lb0 + pc0 * 16), voff, 0);
        } else {
          const int hp = pc - DYQ, hv = hp >> 3, q = hp & 7;
          const int hw_ = hv % HW, t_ = hv / HW, hh_ = t_ % HH, hd_ = t_ / HH;
          const int gd = d0 + hd_ - 1, gh = h0 + hh_ - 1, gw = w0 + hw_ - 1;
          if (hp < XQ && gd >= 0 && gd < p.D && gh >= 0 && gh < p.H && gw >= 0 && gw < p.W && xc + q * 4 < xs)
            voff = (uint32_t)(((((n * p.D + gd) * p.H + gh) * p.W + gw) * xs + xc + q * 4) * 4);
          dma16(xr, __builtin_amdgcn_readfirstlane(lb0 + Tr::RAWDY + (pc0 - DYQ) * 16), voff, 0);
        }
      }
    } else {
      (void)b;
    }
  };
  auto split_raw = [&](char* buf) __attribute__((always_inline)) {
    if constexpr (kX6) {
      const char* raw = wlds + Tr::NPART * BUFBYTES;
      constexpr int DYQ = Tr::BV * 16;
      const int XQ = HV * 8;
      for (int pc = tid; pc < DYQ + XQ; pc += kWThreads) {
        const bool isdy = pc < DYQ;
        const f32x4_t v = *reinterpret_cast<const f32x4_t*>(isdy ? raw + pc * 16 : raw + Tr::RAWDY + (pc - DYQ) * 16);
        const int off = isdy ? dy_off_bf16(pc >> 4, (pc & 15) * 4) : DYBYTES + (pc - DYQ) * 8;
        const float f[8] = {v[0], v[1], v[2], v[3], 0.f, 0.f, 0.f, 0.f};
        u32x4_t h, m, l;
        split3x8(f, h, m, l);
        *reinterpret_cast<u32x2_t*>(buf + off) = (u32x2_t){h[0], h[1]};
        *reinterpret_cast<u32x2_t*>(buf + BUFBYTES + off) = (u32x2_t){m[0], m[1]};
        *reinterpret_cast<u32x2_t*>(buf + 2 * BUFBYTES + off) = (u32x2_t){l[0], l[1]};
      }
    } else {
      (void)buf;
    }
  };

  // per-lane voxel-row helpers for the k index (voxel inside the box)
  auto halo_row = [&](int r) {
    const int rd = r >> (lbh_ + lbw_), rh = (r >> lbw_) & (bh - 1), rw = r & (bw - 1);
    return (rd * HH + rh) * HW + rw;
  };

  // generic box: one 16-voxel k-step at a time.  x3: the lo tiles sit BUFBYTES past the hi
  // tiles; per (co tile, tap) hi*hi + lo*hi + hi*lo
  auto compute = [&](const char* buf) {
    const char* xb = buf + DYBYTES;
#pragma unroll 2
    for (int k0 = 0; k0 < boxvol; k0 += Tr::KV) {
      const int g = (lane >> 4) & 1, qq = (lane & 15) >> 2, pp = lane & 3;
      auto frag = [](const char* base, int o0, int o1) __attribute__((always_inline)) {
        const s16x4_t l = tr_read(base, o0), h = tr_read(base, o1);
        return (s16x8_t){l[0], l[1], l[2], l[3], h[0], h[1], h[2], h[3]};
      };
      if constexpr (kX6) {
        // 8 voxels per k-step, both K halves over the same voxels from different parts:
        // A1 = [dy h | dy m], A2 = [dy h | dy l]; B1 = [x h | x h], B2 = [x m | x h],
        // B3 = [x l | x m]; A1.B1 + A2.B2 + A1.B3 = hh + mh + hm + lh + hl + mm
        const int v_a = k0 + qq;
        const char* dA1 = buf + hsel * BUFBYTES;
        const char* dA2 = buf + hsel * 2 * BUFBYTES;
        s16x8_t a1[2], a2[2];
#pragma unroll
        for (int ct = 0; ct < 2; ++ct) {
          const int co = ct * 32 + g * 16 + pp * 4;
          const int o0 = dy_off_bf16(v_a, co), o1 = dy_off_bf16(v_a + 4, co);
          a1[ct] = frag(dA1, o0, o1);
          a2[ct] = frag(dA2, o0, o1);
        }
        const int hr0 = halo_row(v_a), hr1 = halo_row(v_a + 4);
        const int ci = g * 16 + pp * 4;
        if constexpr (pack4) {
          if (wave < 7) {
            // the lane's 4 columns g 16 + pp 4 .. + 3 = tap 2 g + pp / 2 of the group, channels
            // (pp & 1) 4 .. + 3 (tap 27 of the last group reads tap 26; its column is dropped)
            const int tap = min(4 * wave + 2 * g + (pp >> 1), 26);
            const int kd = tap / 9, kh = (tap / 3) % 3, kw = tap % 3;
            const int off = (kd * HH + kh) * HW + kw;
            const int o0 = (hr0 + off) * Tr::XROW + (pp & 1) * 8, o1 = (hr1 + off) * Tr::XROW + (pp & 1) * 8;
            const s16x8_t b1 = frag(xb, o0, o1);
            const s16x8_t b2 = frag(xb + (hsel ? 0 : BUFBYTES), o0, o1);
            const s16x8_t b3 = frag(xb + (hsel ? BUFBYTES : 2 * BUFBYTES), o0, o1);
#pragma unroll
            for (int ct = 0; ct < 2; ++ct) {
              acc[4 * ct] = mfma(a1[ct], b1, acc[4 * ct]);
              acc[4 * ct] = mfma(a2[ct], b2, acc[4 * ct]);
              acc[4 * ct] = mfma(a1[ct], b3, acc[4 * ct]);
            }
          }
          continue;
        }
        const char* xb1 = xb;                                     // B1: h | h
        const char* xb2 = xb + (hsel ? 0 : BUFBYTES);            // B2: m | h
        const char* xb3 = xb + (hsel ? BUFBYTES : 2 * BUFBYTES);  // B3: l | m
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (owned(j)) {
            const int tap = tapof(j);
            const int kd = tap / 9, kh = (tap / 3) % 3, kw = tap % 3;
            const int off = (kd * HH + kh) * HW + kw;
            const int o0 = (hr0 + off) * Tr::XROW + ci * 2, o1 = (hr1 + off) * Tr::XROW + ci * 2;
            const s16x8_t b1 = frag(xb1, o0, o1), b2 = frag(xb2, o0, o1), b3 = frag(xb3, o0, o1);
#pragma unroll
            for (int ct = 0; ct < 2; ++ct) {
              acc[4 * ct + j] = mfma(a1[ct], b1, acc[4 * ct + j]);
              acc[4 * ct + j] = mfma(a2[ct], b2, acc[4 * ct + j]);
              acc[4 * ct + j] = mfma(a1[ct], b3, acc[4 * ct + j]);
            }
          }
        }
        continue;
      }
      const int v_a = k0 + 8 * hsel + qq;
      s16x8_t a2[2], a2l[2];
#pragma unroll
      for (int ct = 0; ct < 2; ++ct) {
        const int co = ct * 32 + g * 16 + pp * 4;
        a2[ct] = frag(buf, dy_off_bf16(v_a, co), dy_off_bf16(v_a + 4, co));
        if constexpr (kX3) a2l[ct] = frag(buf + BUFBYTES, dy_off_bf16(v_a, co), dy_off_bf16(v_a + 4, co));
      }
      const int hr0 = LBW >= 4 ? halo_row(k0) + 8 * hsel + qq : halo_row(v_a);
      const int hr1 = LBW >= 4 ? hr0 + 4 : halo_row(v_a + 4);
      const int ci = g * 16 + pp * 4;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (owned(j)) {
          const int tap = tapof(j);
          const int kd = tap / 9, kh = (tap / 3) % 3, kw = tap % 3;
          const int off = (kd * HH + kh) * HW + kw;
          const int o0 = (hr0 + off) * Tr::XROW + ci * 2, o1 = (hr1 + off) * Tr::XROW + ci * 2;
          const s16x8_t b = frag(xb, o0, o1);
          acc[j] = mfma(a2[0], b, acc[j]);
          acc[4 + j] = mfma(a2[1], b, acc[4 + j]);
          if constexpr (kX3) {
            const s16x8_t bl = frag(xb + BUFBYTES, o0, o1);
            acc[j] = mfma(a2l[0], b, acc[j]);
            acc[4 + j] = mfma(a2l[1], b, acc[4 + j]);
            acc[j] = mfma(a2[0], bl, acc[j]);
            acc[4 + j] = mfma(a2[1], bl, acc[4 + j]);
          }
        }
      }
    }
  };

  // bf16 with a compile-time box (w = 8 or 16): the k loop fully unrolled.  Every fragment
  // address is a per-lane base (per box buffer) + an immediate: the dy half swap depends on the
  // lane's voxel inside a 16-voxel step only, a step starts a w-row, and the lane's voxels
  // (vl, vl + 4) lie in one w-row (vl % 8 < 4), so its halo rows are a lane constant plus the
  // step's compile-time row.  The
  // fragments of step s + 1 are read while step s's MFMAs run (two register sets), so the
  // LDS latency is behind the MFMAs instead of in front of each pair.  Taps wave + 8 j, j < 3
  // for every wave; the fourth (waves 0-2: taps 24-26) in a uniform branch at the step's end,
  // its fragment also one step ahead (one code path: no per-variant register allocation).
  auto compute_fixed = [&](const char* buf, auto&& mid, auto&& stage) __attribute__((always_inline)) {
    constexpr int LD = LBW >= 2 ? LBD : 0, LH = LBW >= 2 ? LBH : 0, LW = LBW >= 2 ? LBW : 4;
    constexpr int HHc = (1 << LH) + 2, HWc = (1 << LW) + 2;
    constexpr int NK = (1 << (LD + LH + LW)) / 16;
    // halo rows between a lane's two voxels vl and vl + 4: the same w-row (w >= 8: vl % 8 < 4)
    // or, at w = 4, the next h-row (LH >= 2: a 16-voxel step stays inside one d-plane)
    static_assert(LW >= 3 || (LW == 2 && LH >= 2), "compile-time wgrad box");
    constexpr int D4 = LW >= 3 ? 4 : HWc;
    const int g = (lane >> 4) & 1, qq = (lane & 15) >> 2, pp = lane & 3;
    const int vl = 8 * hsel + qq;  // the lane's first voxel inside a step
    const int vrow = (vl >> LW) * HWc + (vl & ((1 << LW) - 1));  // its halo row offset
    const char* ab0 = buf + dy_off_bf16(vl, g * 16 + pp * 4);
    const char* ab1 = buf + dy_off_bf16(vl, 32 + g * 16 + pp * 4);
    const char* bb[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int tap = tapof(j);
      const int kd = tap / 9, kh = (tap / 3) % 3, kw = tap % 3;
      bb[j] = buf + DYBYTES + (vrow + (kd * HHc + kh) * HWc + kw) * Tr::XROW + (g * 16 + pp * 4) * 2;
    }
    auto cat = [](s16x4_t lo, s16x4_t hi) __attribute__((always_inline)) {
      return (s16x8_t){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    };
    auto hro = [](int s) __attribute__((always_inline)) {  // the step's first halo row (w = 0)
      const int v0 = 16 * s, rd = v0 >> (LH + LW), rh = (v0 >> LW) & ((1 << LH) - 1);
      return (rd * HHc + rh) * HWc * Tr::XROW;
    };
    s16x8_t fa[2][2], fb[2][3], f3[2];
    auto load = [&](int s, int set) __attribute__((always_inline)) {
      fa[set][0] = cat(tr_read(ab0, s * 2048), tr_read(ab0, s * 2048 + 512));
      fa[set][1] = cat(tr_read(ab1, s * 2048), tr_read(ab1, s * 2048 + 512));
#pragma unroll
      for (int j = 0; j < NJ; ++j) fb[set][j] = cat(tr_read(bb[j], hro(s)), tr_read(bb[j], hro(s) + D4 * Tr::XROW));
    };
    auto load3 = [&](int s, int set) __attribute__((always_inline)) {
      f3[set] = cat(tr_read(bb[3], hro(s)), tr_read(bb[3], hro(s) + D4 * Tr::XROW));
    };
    load(0, 0);
    if (four) load3(0, 0);
    static_for<NK>([&](auto sc) __attribute__((always_inline)) {
      constexpr int s = decltype(sc)::value, cs = s & 1, ns = cs ^ 1;
      stage(sc);  // the next box's halo pieces of this step (their address VALU under the MFMAs)
      if constexpr (s == NK / 2) mid();  // BNIN: the next box's BN apply under this box's MFMAs
      if constexpr (s + 1 < NK) load(s + 1, ns);
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        acc[j] = mfma(fa[cs][0], fb[cs][j], acc[j]);
        acc[4 + j] = mfma(fa[cs][1], fb[cs][j], acc[4 + j]);
      }
      if (four) {
        if constexpr (s + 1 < NK) load3(s + 1, ns);
        acc[3] = mfma(fa[cs][0], f3[cs], acc[3]);
        acc[7] = mfma(fa[cs][1], f3[cs], acc[7]);
      }
    });
  };
  // K16: 32-voxel steps; lane (G = lane / 16, q, pp) reads voxels 8 G + q and 8 G + q + 4 of a
  // step (one w-row, or two adjacent h-rows at w = 4), A = dy^T rows co 16 c + 4 pp.., B = x
  // columns ci 16 t + 4 pp.. of the tap's halo rows; MFMAs walk co tile c outermost.
  auto compute_fixed16 = [&](const char* buf, auto&& mid, auto&& stage) __attribute__((always_inline)) {
    constexpr int LD = LBW >= 2 ? LBD : 0, LH = LBW >= 2 ? LBH : 0, LW = LBW >= 2 ? LBW : 4;
    constexpr int HHc = (1 << LH) + 2, HWc = (1 << LW) + 2;
    constexpr int NK = (1 << (LD + LH + LW)) / 32;
    static_assert(LW >= 3 || (LW == 2 && LH >= 3), "K16 box: a 32-voxel step stays in one d-plane");
    constexpr int D4 = LW >= 3 ? 4 : HWc;
    const int G4 = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
    const int vl = 8 * G4 + q;
    const int vrow = (vl >> LW) * HWc + (vl & ((1 << LW) - 1));
    const char* ab[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) ab[c] = buf + dy_off_bf16(vl, c * 16 + pp * 4);
    const char* bb[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int tap = tapof(j);
      const int kd = tap / 9, kh = (tap / 3) % 3, kw = tap % 3;
      bb[j] = buf + DYBYTES + (vrow + (kd * HHc + kh) * HWc + kw) * Tr::XROW + pp * 8;
    }
    auto cat = [](s16x4_t lo, s16x4_t hi) __attribute__((always_inline)) {
      return (s16x8_t){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    };
    auto hro = [](int s) __attribute__((always_inline)) {
      const int v0 = 32 * s, rd = v0 >> (LH + LW), rh = (v0 >> LW) & ((1 << LH) - 1);
      return (rd * HHc + rh) * HWc * Tr::XROW;
    };
    // one register set per operand: co tile c's A fragment of step s + 1 is read right after
    // c's MFMAs of step s (a whole step of slack); tap j's B fragments after their last use
    // (c = 3), a few MFMAs before the next step needs them (the other wave of the SIMD covers)
    s16x8_t fa[4], fb[4][2];
    auto loadA = [&](int s, int c) __attribute__((always_inline)) {
      fa[c] = cat(tr_read(ab[c], s * 4096), tr_read(ab[c], s * 4096 + 512));
    };
    auto loadB = [&](int s, int j) __attribute__((always_inline)) {
#pragma unroll
      for (int t = 0; t < 2; ++t)
        fb[j][t] = cat(tr_read(bb[j], hro(s) + t * 32), tr_read(bb[j], hro(s) + D4 * Tr::XROW + t * 32));
    };
#pragma unroll
    for (int c = 0; c < 4; ++c) loadA(0, c);
#pragma unroll
    for (int j = 0; j < NJ; ++j) loadB(0, j);
    if (four) loadB(0, 3);
    static_for<NK>([&](auto sc) __attribute__((always_inline)) {
      constexpr int s = decltype(sc)::value;
      stage(sc);
      if constexpr (s == NK / 2) mid();  // BNIN: the next box's BN apply under this box's MFMAs
      static_for<4>([&](auto ccc) __attribute__((always_inline)) {
        constexpr int c = decltype(ccc)::value;
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
#pragma unroll
          for (int t = 0; t < 2; ++t) acc16[j][c][t] = mfma16(fa[c], fb[j][t], acc16[j][c][t]);
          if constexpr (c == 3 && s + 1 < NK) loadB(s + 1, j);
        }
        if (four) {
#pragma unroll
          for (int t = 0; t < 2; ++t) acc16[3][c][t] = mfma16(fa[c], fb[3][t], acc16[3][c][t]);
          if constexpr (c == 3 && s + 1 < NK) loadB(s + 1, 3);
        }
        if constexpr (s + 1 < NK) loadA(s + 1, c);
      });
    });
  };
  // mid(): work placed halfway through the box's MFMA steps (compute_fixed), or after them
  // stage(s): called at the start of every k-step of the compile-time-box loops
  constexpr bool kSpread = !kX3 && !kX6 && LBW >= 2;
  auto compute_box = [&](const char* buf, auto&& mid, auto&& stage) __attribute__((always_inline)) {
    if constexpr (K16) {
      compute_fixed16(buf, mid, stage);
    } else if constexpr (kSpread) {
      compute_fixed(buf, mid, stage);
    } else {
      compute(buf);
      mid();
    }
  };
  auto nomid = []() __attribute__((always_inline)) {};
  auto nostage = [](auto) __attribute__((always_inline)) {};

  // bf16 hot path: both tiles arrive by buffer LDS-DMA (no register staging); the next box
  // streams in while this one computes.  The dy tile keeps dy_off_bf16's half swap (applied
  // to the source address); each wave instruction is all-dy or all-halo (2048 dy pieces);
  // out-of-range pieces read zeros.
  // BNIN: bit i = piece i of this thread is a real (in-range) x-halo piece
  // piece i (16 B; i < MAXP) of this thread for the box at (n, d0, h0, w0) into buf; returns
  // bit i when it is a real (in-range) x-halo piece (BNIN)
  auto stage_piece = [&](char* buf, int i, int n, int d0, int h0, int w0) -> uint32_t {
    const int pc0 = (tid & ~63) + i * kWThreads;  // wave-uniform first piece
    if (pc0 >= DYP + XP) return 0u;
    const uint32_t lb0 = lds_addr(buf);
    const int pc = pc0 + lane;
    uint32_t voff = kOOB;
    if (pc0 < DYP) {
      const int r = pc >> 3, q = pc & 7;
      const int ql = q ^ (((r >> 1) & 1) << 2);
      if (r < boxvol) {
        const int rd = r >> (lbh_ + lbw_), rh = (r >> lbw_) & (bh - 1), rw = r & (bw - 1);
        const int gd = d0 + rd, gh = h0 + rh, gw = w0 + rw;
        if (gd < p.D && gh < p.H && gw < p.W)
          voff = (uint32_t)(((((n * p.D + gd) * p.H + gh) * p.W + gw) * p.Cout + co_base + ql * 8) * 2);
      }
      if constexpr (WGRAD_ABL & 16) { asm volatile("" ::"v"(voff)); voff = kOOB; }
      if constexpr (WGRAD_ABL & 32) voff = (uint32_t)(pc * 16);
      dma16(buffer_desc(p.dy, p.dybytes), __builtin_amdgcn_readfirstlane(lb0 + pc0 * 16), voff, 0);
      return 0u;
    }
    const bool first = ci_base < p.c0;  // a 32-channel block lies in one source
    const int xs = first ? p.c0 : p.c1, xc = first ? ci_base : ci_base - p.c0;
    const int hp = pc - DYP;
    const int hv = hp >> 2, q = hp & 3;
    const int hw_ = hv % HW, t_ = hv / HW, hh_ = t_ % HH, hd_ = t_ / HH;
    const int gd = d0 + hd_ - 1, gh = h0 + hh_ - 1, gw = w0 + hw_ - 1;
    if (hp < XP && gd >= 0 && gd < p.D && gh >= 0 && gh < p.H && gw >= 0 && gw < p.W && xc + q * 8 < xs)
      voff = (uint32_t)(((((n * p.D + gd) * p.H + gh) * p.W + gw) * xs + xc + q * 8) * 2);
    if constexpr (WGRAD_ABL & 16) { asm volatile("" ::"v"(voff)); voff = kOOB; }
    if constexpr (WGRAD_ABL & 32) voff = (uint32_t)(pc * 16);
    dma16(buffer_desc(first ? p.x0 : p.x1, first ? p.x0bytes : p.x1bytes),
          __builtin_amdgcn_readfirstlane(lb0 + DYBYTES + (pc0 - DYP) * 16), voff, 0);
    return voff != kOOB ? 1u << i : 0u;
  };
  // compile-time boxes: each piece's source offset relative to its box origin does not depend
  // on the box, so it is formed once (prel: elements past the box-origin voxel's first channel,
  // pco: the halo coordinates hd | hh << 8 | hw << 16 of an x piece, -1 for padding pieces);
  // a box then costs one add per piece, plus 3 compares on boxes that touch the volume's border.
  // (Measured neutral here -- 819 vs 823-832 us at level 0, profiles/r5_wgrad_prel_abl.txt:
  // with two waves per SIMD the VALU already hid under the other wave's MFMAs; what the
  // fixed-address ablation gained, profiles/r5_wgrad_addr_abl.txt, was L2 hits, not arithmetic.)
  int prel[kSpread ? MAXP : 1], pco[kSpread ? MAXP : 1];
  if constexpr (kSpread) {
    const bool first = ci_base < p.c0;
    const int xs = first ? p.c0 : p.c1, xc = first ? ci_base : ci_base - p.c0;
#pragma unroll
    for (int i = 0; i < MAXP; ++i) {
      const int pc = (tid & ~63) + i * kWThreads + lane;
      if ((tid & ~63) + i * kWThreads < DYP) {
        const int r = pc >> 3, q = pc & 7;
        const int ql = q ^ (((r >> 1) & 1) << 2);
        const int rd = r >> (lbh_ + lbw_), rh = (r >> lbw_) & (bh - 1), rw = r & (bw - 1);
        prel[i] = ((rd * p.H + rh) * p.W + rw) * p.Cout + co_base + ql * 8;
        pco[i] = r < boxvol ? (rd | (rh << 8) | (rw << 16)) : -1;
      } else {
        const int hp = pc - DYP, hv = hp >> 2, q = hp & 3;
        const int hw_ = hv % HW, t_ = hv / HW, hh_ = t_ % HH, hd_ = t_ / HH;
        prel[i] = (((hd_ - 1) * p.H + (hh_ - 1)) * p.W + (hw_ - 1)) * xs + xc + q * 8;
        pco[i] = (hp < XP && xc + q * 8 < xs) ? (hd_ | (hh_ << 8) | (hw_ << 16)) : -1;
      }
    }
  }
  // piece i of the box at (n, d0, h0, w0): `inner` = the box and its halo lie inside the volume
  auto stage_piece_fast = [&](char* buf, int i, int n, int d0, int h0, int w0, bool inner) -> uint32_t {
    const int pc0 = (tid & ~63) + i * kWThreads;
    if (pc0 >= DYP + XP) return 0u;
    const uint32_t lb0 = lds_addr(buf);
    const int c = pco[i];
    const long vb = ((long)(n * p.D + d0) * p.H + h0) * p.W + w0;
    uint32_t voff;
    if (pc0 < DYP) {
      voff = (uint32_t)((vb * p.Cout + prel[i]) * 2);
      if (c < 0) voff = kOOB;
      else if (!inner && (d0 + (c & 255) >= p.D || h0 + ((c >> 8) & 255) >= p.H || w0 + (c >> 16) >= p.W)) voff = kOOB;
      dma16(buffer_desc(p.dy, p.dybytes), __builtin_amdgcn_readfirstlane(lb0 + pc0 * 16), voff, 0);
      return 0u;
    }
    const bool first = ci_base < p.c0;
    const int xs = first ? p.c0 : p.c1;
    voff = (uint32_t)((vb * xs + prel[i]) * 2);
    if (c < 0) {
      voff = kOOB;
    } else if (!inner) {
      const int gd = d0 + (c & 255) - 1, gh = h0 + ((c >> 8) & 255) - 1, gw = w0 + (c >> 16) - 1;
      if ((unsigned)gd >= (unsigned)p.D || (unsigned)gh >= (unsigned)p.H || (unsigned)gw >= (unsigned)p.W) voff = kOOB;
    }
    if constexpr (WGRAD_ABL & 16) { asm volatile("" ::"v"(voff)); voff = kOOB; }
    if constexpr (WGRAD_ABL & 32) voff = (uint32_t)((pc0 + lane) * 16);
    dma16(buffer_desc(first ? p.x0 : p.x1, first ? p.x0bytes : p.x1bytes),
          __builtin_amdgcn_readfirstlane(lb0 + DYBYTES + (pc0 - DYP) * 16), voff, 0);
    return voff != kOOB ? 1u << i : 0u;
  };
  // a whole box at once (runtime-geometry kernels and the first box)
  auto stage_dma = [&](char* buf, int b) -> uint32_t {
    uint32_t xm = 0;
    int n, d0, h0, w0;
    box_origin(b, n, d0, h0, w0);
    const uint32_t lb0 = lds_addr(buf);
    const bool first = ci_base < p.c0;  // a 32-channel block lies in one source
    const i32x4_t xr = buffer_desc(first ? p.x0 : p.x1, first ? p.x0bytes : p.x1bytes);
    const i32x4_t dr = buffer_desc(p.dy, p.dybytes);
    const int xs = first ? p.c0 : p.c1, xc = first ? ci_base : ci_base - p.c0;
#pragma unroll
    for (int i = 0; i < MAXP; ++i) {
      const int pc0 = (tid & ~63) + i * kWThreads;  // wave-uniform first piece
      if (pc0 >= DYP + XP) break;
      const int pc = pc0 + lane;
      uint32_t voff = kOOB;
      if (pc0 < DYP) {
        const int r = pc >> 3, q = pc & 7;
        const int ql = q ^ (((r >> 1) & 1) << 2);
        if (r < boxvol) {
          const int rd = r >> (lbh_ + lbw_), rh = (r >> lbw_) & (bh - 1), rw = r & (bw - 1);
          const int gd = d0 + rd, gh = h0 + rh, gw = w0 + rw;
          if (gd < p.D && gh < p.H && gw < p.W)
            voff = (uint32_t)(((((n * p.D + gd) * p.H + gh) * p.W + gw) * p.Cout + co_base + ql * 8) * 2);
        }
        dma16(dr, __builtin_amdgcn_readfirstlane(lb0 + pc0 * 16), voff, 0);
      } else {
        const int hp = pc - DYP;
        const int hv = hp >> 2, q = hp & 3;
        const int hw_ = hv % HW, t_ = hv / HW, hh_ = t_ % HH, hd_ = t_ / HH;
        const int gd = d0 + hd_ - 1, gh = h0 + hh_ - 1, gw = w0 + hw_ - 1;
        if (hp < XP && gd >= 0 && gd < p.D && gh >= 0 && gh < p.H && gw >= 0 && gw < p.W && xc + q * 8 < xs)
          voff = (uint32_t)(((((n * p.D + gd) * p.H + gh) * p.W + gw) * xs + xc + q * 8) * 2);
        dma16(xr, __builtin_amdgcn_readfirstlane(lb0 + DYBYTES + (pc0 - DYP) * 16), voff, 0);
        if (voff != kOOB) xm |= 1u << i;
      }
    }
    return xm;
  };
  // BNIN: this thread's landed x pieces of buffer buf in place (every piece of a thread has
  // channel group q = tid & 3: DYP and the 512-piece rounds are multiples of 4)
  float* bnt = reinterpret_cast<float*>(wlds + Tr::NBUF * BUFBYTES);
  auto bn_x = [&](char* buf, uint32_t xm) {
    const int q = tid & 3;
    const f32x4_t s0 = *reinterpret_cast<const f32x4_t*>(bnt + q * 8), s1 = *reinterpret_cast<const f32x4_t*>(bnt + q * 8 + 4);
    const f32x4_t h0 = *reinterpret_cast<const f32x4_t*>(bnt + 32 + q * 8);
    const f32x4_t h1 = *reinterpret_cast<const f32x4_t*>(bnt + 32 + q * 8 + 4);
    const float sc[8] = {s0[0], s0[1], s0[2], s0[3], s1[0], s1[1], s1[2], s1[3]};
    const float sh[8] = {h0[0], h0[1], h0[2], h0[3], h1[0], h1[1], h1[2], h1[3]};
#pragma unroll
    for (int i = 0; i < MAXP; ++i) {
      if (!((xm >> i) & 1)) continue;
      u32x4_t* v = reinterpret_cast<u32x4_t*>(buf + DYBYTES + (tid + i * kWThreads - DYP) * 16);
      u32x4_t x = *v;
#pragma unroll
      for (int k = 0; k < 4; ++k)
        x[k] = pack_bf16x2(bn_relu1(__uint_as_float(x[k] << 16), sc[2 * k], sh[2 * k]),
                           bn_relu1(__uint_as_float(x[k] & 0xffff0000u), sc[2 * k + 1], sh[2 * k + 1]));
      *v = x;
    }
  };
  if constexpr (BNIN) {
    if (tid < 32) {
      const int c = ci_base + tid;
      bnt[tid] = c < p.Cin ? p.isc[c] : 0.f;
      bnt[32 + tid] = c < p.Cin ? p.ish[c] : 0.f;
    }
    __syncthreads();
  }

  if (!kX6 && b_beg < b_end && p.dma) {
    if constexpr (Tr::NBUF == 2) {
      uint32_t xm = stage_dma(wlds, b_beg);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if constexpr (BNIN) bn_x(wlds, xm);
      __syncthreads();
      for (int b = b_beg; b < b_end; ++b) {
        const int cur = (b - b_beg) & 1;
        const bool nxt = b + 1 < b_end && !(WGRAD_ABL & 2);
        char* nbuf = wlds + (cur ^ 1) * BUFBYTES;
        // compile-time boxes: the next box's pieces are issued PPS per k-step over the first
        // SPW steps, so their address arithmetic runs on the VALU beside this box's MFMAs
        // instead of in a block before them (where both waves of a SIMD stalled the MFMA pipe
        // together); they land long before the box-end wait (BNIN: before its apply at NK / 2)
        int n1 = 0, d1 = 0, h1 = 0, w1 = 0;
        bool inner1 = false;
        if constexpr (kSpread && !(WGRAD_ABL & 4)) {
          if (nxt) {
            box_origin(b + 1, n1, d1, h1, w1);
            inner1 = d1 >= 1 && d1 + bd < p.D && h1 >= 1 && h1 + bh < p.H && w1 >= 1 && w1 + bw < p.W;
          }
          xm = 0;
        } else if (nxt) {
          xm = stage_dma(nbuf, b + 1);
        }
        auto stage = [&](auto sc) __attribute__((always_inline)) {
          if constexpr (kSpread) {
            constexpr int st = decltype(sc)::value;
            constexpr int NKc = (1 << (LBD + LBH + LBW)) / (K16 ? 32 : 16);
            constexpr int SPW = BNIN ? NKc / 4 : NKc / 2;
            constexpr int PPS = (MAXP + SPW - 1) / SPW;
            if constexpr (st * PPS < MAXP) {
              if (nxt) {
#pragma unroll
                for (int k = 0; k < PPS; ++k)
                  if (st * PPS + k < MAXP) xm |= stage_piece_fast(nbuf, st * PPS + k, n1, d1, h1, w1, inner1);
              }
            }
          }
        };
        if constexpr (BNIN) {
          // this thread's pieces of box b + 1 have landed once its vmcnt drains (LDS-DMA
          // completion is per wave); nobody reads buffer cur ^ 1 before the barrier below
          compute_box(wlds + cur * BUFBYTES, [&]() __attribute__((always_inline)) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (b + 1 < b_end) bn_x(nbuf, xm);
          }, stage);
        } else if constexpr (!(WGRAD_ABL & 4)) {
          compute_box(wlds + cur * BUFBYTES, nomid, stage);
        }
        if constexpr (!(WGRAD_ABL & 8)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
      }
    }
  } else if (kX6 && b_beg < b_end && p.dma) {
    if constexpr (kX6) {
      // fp32 build (bf16x6) with LDS-DMA: box b + 1 streams into the fp32 staging buffer while
      // box b's MFMAs run on its split tiles; between boxes every thread splits its pieces of
      // the landed box into the h / m / l tiles (the values stage_x3 writes)
      stage_raw(b_beg);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      for (int b = b_beg; b < b_end; ++b) {
        split_raw(wlds);
        __syncthreads();
        if (b + 1 < b_end) stage_raw(b + 1);
        compute(wlds);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
      }
    }
  } else if (b_beg < b_end) {
    if constexpr (Tr::NBUF == 2) {
      stage_load(b_beg);
      stage_store(wlds);
      __syncthreads();
      for (int b = b_beg; b < b_end; ++b) {
        const int cur = (b - b_beg) & 1;
        if (b + 1 < b_end) stage_load(b + 1);
        compute_box(wlds + cur * BUFBYTES, nomid, nostage);
        if (b + 1 < b_end) stage_store(wlds + (cur ^ 1) * BUFBYTES);
        __syncthreads();
      }
    } else {
      // fp32 build: synchronous staging (all of a box's loads in flight, split on the way
      // into LDS), then the box's MFMAs
      for (int b = b_beg; b < b_end; ++b) {
        __syncthreads();
        stage_x3(wlds, b);
        __syncthreads();
        compute(wlds);
      }
    }
  }

  // flush: C[row = co][col = ci] of tap -> this split's partial row dwt[split][tap][co][ci]
  // with plain stores (two 128-B row segments per instruction); the splits are summed in a
  // fixed order by wgrad_group_sum_kernel / wgrad_reduce_kernel.  (fp32 atomics from every
  // split into one [27][Cout][Cin] image serialised on the contended addresses: 2-4x the
  // kernel's own time at level 0.)
  float* prow = p.dwt + (long)split * 27 * p.Cout * p.Cin;
  {
    if (p.direct) {
      // one split: no partial rows to reduce.  Per 32-row co half, the workgroup's
      // [32 co][32 ci][27 taps] tile is transposed through LDS (the staging buffers are free)
      // and added to the contiguous [ci][27] runs of the torch-layout dw.
      float* tile = reinterpret_cast<float*>(wlds);
      const int nci = min(32, p.cw - ci_base);
      for (int ct = 0; ct < 2; ++ct) {
        __syncthreads();
        if constexpr (pack4) {
          const int tap = 4 * wave + ((lane & 31) >> 3);
          if (wave < 7 && tap < 27)
#pragma unroll
            for (int e = 0; e < 16; ++e) {
              const int col = (e & 3) + 8 * (e >> 2) + 4 * hsel;
              tile[(col * 32 + (lane & 7)) * 27 + tap] = acc[ct * 4][e];
            }
        } else if constexpr (K16) {
          // acc16[j][c][t] element e: co 16 c + 4 (lane / 16) + e, ci 16 t + lane % 16
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            if (!owned(j)) continue;
            const int tap = tapof(j);
#pragma unroll
            for (int cc = 0; cc < 2; ++cc)
#pragma unroll
              for (int t = 0; t < 2; ++t)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                  const int col = cc * 16 + 4 * (lane >> 4) + e;
                  tile[(col * 32 + t * 16 + (lane & 15)) * 27 + tap] = acc16[j][2 * ct + cc][t][e];
                }
          }
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            if (!owned(j)) continue;
            const int tap = tapof(j);
#pragma unroll
            for (int e = 0; e < 16; ++e) {
              const int col = (e & 3) + 8 * (e >> 2) + 4 * hsel;
              tile[(col * 32 + (lane & 31)) * 27 + tap] = acc[ct * 4 + j][e];
            }
          }
        }
        __syncthreads();
        if (TG) {
          // this group's taps only (the other group's workgroup writes the rest of each run)
          for (int i = tid; i < 32 * 32 * 27; i += kWThreads) {
            const int col = i / 864, r = i % 864, tap = r % 27;
            const int co = co_base + ct * 32 + col;
            if (co < p.Cout && r < nci * 27 && (tap >= 16) == (tgrp == 1)) {
              float* d = p.dw + ((long)co * p.cw + ci_base) * 27 + r;
              *d = p.store ? tile[i] : *d + tile[i];
            }
          }
        } else if (nci == 32) {
          // whole 32 x 864-float runs: 16-B read-modify-writes, all of a thread's loads in
          // flight before the first add (a dependent load -> add -> store chain per element
          // made the deep levels latency-bound)
          constexpr int kQ = 32 * 216, kPer = (kQ + kWThreads - 1) / kWThreads;
          f32x4_t g[kPer];
#pragma unroll
          for (int k = 0; k < kPer; ++k) {
            const int q4 = tid + k * kWThreads, row = q4 / 216, q = q4 % 216;
            g[k] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
            if (q4 < kQ && !p.store)  // store: plain stores, nothing to read back
              g[k] = *reinterpret_cast<const f32x4_t*>(p.dw + ((long)(co_base + ct * 32 + row) * p.cw + ci_base) * 27 + 4 * q);
          }
#pragma unroll
          for (int k = 0; k < kPer; ++k) {
            const int q4 = tid + k * kWThreads, row = q4 / 216, q = q4 % 216;
#if WGRAD_ABL & 1  // ablation build: the flush's global stores dropped
            const f32x4_t o = g[k] + *reinterpret_cast<const f32x4_t*>(tile + row * 864 + 4 * q);
            if (q4 < kQ && o[0] == 1.2345e30f)
              *reinterpret_cast<f32x4_t*>(p.dw + ((long)(co_base + ct * 32 + row) * p.cw + ci_base) * 27 + 4 * q) = o;
#else
            if (q4 < kQ)
              *reinterpret_cast<f32x4_t*>(p.dw + ((long)(co_base + ct * 32 + row) * p.cw + ci_base) * 27 + 4 * q) =
                  g[k] + *reinterpret_cast<const f32x4_t*>(tile + row * 864 + 4 * q);
#endif
          }
        } else {
          for (int i = tid; i < 32 * 32 * 27; i += kWThreads) {
            const int col = i / 864, r = i % 864;  // r = ci * 27 + tap
            const int co = co_base + ct * 32 + col;
            if (co < p.Cout && r < nci * 27) {
              float* d = p.dw + ((long)co * p.cw + ci_base) * 27 + r;
              *d = p.store ? tile[i] : *d + tile[i];
            }
          }
        }
      }
      return;
    }
    if constexpr (pack4) {
      const int tap = 4 * wave + ((lane & 31) >> 3), ci = ci_base + (lane & 7);
      if (wave < 7 && tap < 27 && ci < p.Cin)
#pragma unroll
        for (int ct = 0; ct < 2; ++ct)
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            const int co = co_base + ct * 32 + (e & 3) + 8 * (e >> 2) + 4 * hsel;
            if (co < p.Cout) prow[((long)tap * p.Cout + co) * p.Cin + ci] = acc[ct * 4][e];
          }
      return;
    }
    if constexpr (K16) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (!owned(j)) continue;
        const int tap = tapof(j);
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
          for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const int co = co_base + c * 16 + 4 * (lane >> 4) + e;
              const int ci = ci_base + t * 16 + (lane & 15);
              if (co < p.Cout && ci < p.Cin) prow[((long)tap * p.Cout + co) * p.Cin + ci] = acc16[j][c][t][e];
            }
      }
      return;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (!owned(j)) continue;
      const int tap = tapof(j);
#pragma unroll
      for (int ct = 0; ct < 2; ++ct)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int co = co_base + ct * 32 + (e & 3) + 8 * (e >> 2) + 4 * hsel;
          const int ci = ci_base + (lane & 31);
          if (co < p.Cout && ci < p.Cin) prow[((long)tap * p.Cout + co) * p.Cin + ci] = acc[ct * 4 + j][e];
        }
    }
  }
}

// Weight-gradient split reduction (deterministic, fixed order).  part: S rows of
// E = 27 * Cout * Cin floats ([split][tap][co][ci], Cin = stored channels).
// Stage 1 (S > 16): rows r*16 .. r*16+15 summed in place into row r*16.
__global__ void __launch_bounds__(256) wgrad_group_sum_kernel(float* part, int S, long E) {
  const long e = blockIdx.x * 256L + threadIdx.x;
  if (e >= E) return;
  const int r0 = blockIdx.y * 16, r1 = min(S, r0 + 16);
  part[(long)r0 * E + e] = sum_rows16(part + (long)r0 * E + e, E, r1 - r0);
}
// Stage 2: dw [Cout][Cw][27] (torch OIDHW, the weight's own input-channel count Cw <= Cin;
// stem: 5 of 8) += sum of R rows spaced `stride` rows apart.  Block = (co, 32 channels): the
// [27][32] tiles are read as 128-B rows, transposed through LDS, added to the contiguous
// 32 x 27 run of dw.
__global__ void __launch_bounds__(256) wgrad_reduce_kernel(const float* part, int R, int stride, float* dw,
                                                           int Cout, int Cin, int Cw, int store) {
  __shared__ float tile[27][33];
  const int co = blockIdx.x, ci0 = blockIdx.y * 32;
  const long rstep = (long)stride * 27 * Cout * Cin;
  for (int e = threadIdx.x; e < 27 * 32; e += 256) {
    const int t = e >> 5, c = e & 31, ci = ci0 + c;
    float sum = 0.f;
    if (ci < Cw) {
      sum = sum_rows16(part + ((long)t * Cout + co) * Cin + ci, rstep, R);
    }
    tile[t][c] = sum;
  }
  __syncthreads();
  float* dst = dw + ((long)co * Cw + ci0) * 27;
  const int n = min(32, Cw - ci0) * 27;
  for (int e = threadIdx.x; e < n; e += 256) dst[e] = store ? tile[e % 27][e / 27] : dst[e] + tile[e % 27][e / 27];
}

// Both stages in one launch, same sums bit for bit: the S split rows as G = ceil(S / 16)
// groups of 16, each group summed in row order by one thread, the G group sums then added in
// group order (= wgrad_group_sum_kernel + wgrad_reduce_kernel).  Block = (co, 32 channels) x
// GL group lanes: 256 element lanes (up to 4 of the 864 [27][32] elements each) per group
// lane, all of a group's rows for all of a thread's elements loaded before the first add
// (the two-stage form was a 57 MB pass plus a latency-bound 3.5 MB pass per level-0/1 layer).
// LDS: the [G][27 x 32] group sums.
constexpr int kWredMaxGroups = 16;  // and 16 rows x E floats per group below 2 GB (host check)
static int g_wred_fused = 1;  // 0: the two-stage reduction (A/B, bit-identity test)
template <int GL>
__global__ void __launch_bounds__(256 * GL) wgrad_reduce_fused_kernel(const float* part, int S, float* dw, int Cout,
                                                                      int Cin, int Cw, int store) {
  extern __shared__ float gsum[];  // [G][864]
  constexpr int NE = 27 * 32;
  const int co = blockIdx.x, ci0 = blockIdx.y * 32;
  const long E = 27L * Cout * Cin;
  const int G = (S + 15) / 16;
  const int el = threadIdx.x & 255, gl = threadIdx.x >> 8;
  // 32-bit byte offsets from the group's (uniform) first row: 16 rows x E floats < 2 GB
  uint32_t off[4];
  bool ok[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int e = el + 256 * k, t = e >> 5, c = e & 31;
    ok[k] = e < NE && ci0 + c < Cw;
    off[k] = ok[k] ? (uint32_t)((((long)t * Cout + co) * Cin + ci0 + c) * 4) : 0u;
  }
  const uint32_t rowb = (uint32_t)(E * 4);
  for (int g = gl; g < G; g += GL) {
    const int r0 = g * 16, n = min(16, S - r0);
    // the group's rows through a descriptor: row offset in the SGPR soffset, element offset in
    // one VGPR (a 64-bit address per load held 128 VGPRs of addresses)
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(part + (long)r0 * E), (short)0, (int)(n * rowb), 0x00020000);
    float s[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int h = 0; h < 16; h += 8) {  // 8 rows x 4 elements in flight, added in row order
      float v[4][8];
#pragma unroll
      for (int r = 0; r < 8; ++r)
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if (h + r < n && ok[k])
            v[k][r] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, (int)off[k], (int)((h + r) * rowb), 0));
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int r = 0; r < 8; ++r)
          if (h + r < n && ok[k]) s[k] += v[k][r];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int e = el + 256 * k;
      if (e < NE) gsum[g * NE + e] = s[k];
    }
  }
  __syncthreads();
  float* dst = dw + ((long)co * Cw + ci0) * 27;
  const int n = min(32, Cw - ci0) * 27;
  for (int o = threadIdx.x; o < n; o += 256 * GL) {
    const int c = o / 27, t = o % 27, e = t * 32 + c;
    float s = 0.f;
    for (int g = 0; g < G; ++g) s += gsum[g * NE + e];
    dst[o] = store ? s : dst[o] + s;
  }
}

// master fp32 W[Cout][Cin][27] -> packed T [chunk][27][J][CK]
//   fwd  (flip=0): J = Cout, k-index = ci
//   dgrad(flip=1): J = Cin,  k-index = co, tap mirrored (26 - t)
// One block per (chunk, 8 consecutive j): the 8 x CK x 27 source block is read with unit
// stride into LDS and written back with unit stride in the packed order.
template <typename T, int CK>
__global__ void __launch_bounds__(256) pack_conv3_kernel(const float* w, T* out, int Cout, int Cin, int flip) {
  __shared__ float tile[8][CK][27];
  const int J = flip ? Cin : Cout;
  const int Kdim = flip ? Cout : Cin;
  const int chunk = blockIdx.y;
  const int j0 = blockIdx.x * 8;
  constexpr int E = 8 * CK * 27;
  for (int e = threadIdx.x; e < E; e += 256) {
    int jj, k, t;
    if (!flip) { t = e % 27; k = (e / 27) % CK; jj = e / (27 * CK); }      // w[j][chunk*CK + k][t]
    else { t = e % 27; jj = (e / 27) % 8; k = e / (27 * 8); }             // w[chunk*CK + k][j][t]
    const int kk = chunk * CK + k, j = j0 + jj;
    float v = 0.f;
    if (kk < Kdim && j < J) v = flip ? w[((long)kk * Cin + j) * 27 + t] : w[((long)j * Cin + kk) * 27 + t];
    tile[jj][k][t] = v;
  }
  __syncthreads();
  if constexpr (std::is_same<T, x6_t>::value) {
    // one thread per packed row (t, jj): its 8 k values split once, the 96-B row
    // [h|h] [m|h] [l|m] written as six 16-B stores (consecutive threads: consecutive rows)
    static_assert(CK == 8, "x6 pack rows hold 8 k");
    const int jj = threadIdx.x % 8, t = threadIdx.x / 8;
    if (t < 27 && j0 + jj < J) {
      float f[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) f[k] = flip ? tile[jj][k][26 - t] : tile[jj][k][t];
      u32x4_t h, m, l;
      split3x8(f, h, m, l);
      u32x4_t* o = reinterpret_cast<u32x4_t*>(reinterpret_cast<bf16_t*>(out) + (((long)chunk * 27 + t) * J + j0 + jj) * 48);
      o[0] = h; o[1] = h; o[2] = m; o[3] = h; o[4] = l; o[5] = m;
    }
    return;
  }
  for (int e = threadIdx.x; e < E; e += 256) {
    const int k = e % CK, jj = (e / CK) % 8, t = e / (CK * 8);
    if (j0 + jj >= J) continue;
    const float v = flip ? tile[jj][k][26 - t] : tile[jj][k][t];
    if constexpr (std::is_same<T, x3_t>::value) {
      // split-bf16 pack row [hi k = 0..15 | lo k = 0..15]
      bf16_t* o = reinterpret_cast<bf16_t*>(out) + (((long)chunk * 27 + t) * J + j0 + jj) * 2 * CK;
      const bf16_t hi = f2bf(v);
      o[k] = hi;
      o[CK + k] = f2bf(v - bf2f(hi));
    } else if constexpr (std::is_same<T, x6_t>::value) {
      // three-part pack row: the B fragments [h|h] [m|h] [l|m] (k = 0..7 each half)
      bf16_t* o = reinterpret_cast<bf16_t*>(out) + (((long)chunk * 27 + t) * J + j0 + jj) * 6 * CK;
      const bf16_t h = f2bf(v);
      const float r = v - bf2f(h);
      const bf16_t m = f2bf(r), l = f2bf(r - bf2f(m));
      o[k] = h; o[CK + k] = h;
      o[2 * CK + k] = m; o[3 * CK + k] = h;
      o[4 * CK + k] = l; o[5 * CK + k] = m;
    } else if constexpr (std::is_same<T, bf16_t>::value) {
      out[pack_bf16_off(chunk, t, j0 + jj, k, J)] = Elem<T>::cvt(v);
    } else {
      out[(((long)chunk * 27 + t) * J + j0 + jj) * CK + k] = Elem<T>::cvt(v);
    }
  }
}

// bf16 fast path (Kdim % 32 == 0, J % 8 == 0: every layer but the stem): the same block, read
// as 16-B vectors (the block's source is 8 contiguous 864-float runs (fwd) or 32 contiguous
// 216-float runs (dgrad)) and written as 16-B vectors of 8 packed k.
__global__ void __launch_bounds__(256) pack_conv3_bf16_kernel(const float* w, bf16_t* out, int Cout, int Cin,
                                                              int flip) {
  __shared__ float tile[8][32][27];
  const int J = flip ? Cin : Cout;
  const int chunk = blockIdx.y;
  const int j0 = blockIdx.x * 8;
  for (int e = threadIdx.x; e < 1728; e += 256) {
    int base, run, q;
    if (!flip) {  // w[j0 + jj][chunk*32 .. +32][27]: run jj of 864 floats
      run = e / 216; q = e % 216;
      base = ((j0 + run) * Cin + chunk * 32) * 27;
    } else {      // w[chunk*32 + k][j0 .. j0+8][27]: run k of 216 floats
      run = e / 54; q = e % 54;
      base = ((chunk * 32 + run) * Cin + j0) * 27;
    }
    const f32x4_t v = *reinterpret_cast<const f32x4_t*>(w + base + 4 * q);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int idx = 4 * q + i;
      if (!flip) tile[run][idx / 27][idx % 27] = v[i];
      else tile[idx / 27][run][idx % 27] = v[i];
    }
  }
  __syncthreads();
  for (int g = threadIdx.x; g < 864; g += 256) {
    const int t = g >> 5, jj = (g >> 2) & 7, k8 = (g & 3) * 8;
    const int ts = flip ? 26 - t : t;
    u32x4_t o;
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = pack_bf16x2(tile[jj][k8 + 2 * i][ts], tile[jj][k8 + 2 * i + 1][ts]);
    *reinterpret_cast<u32x4_t*>(out + pack_bf16_off(chunk, t, j0 + jj, k8, J)) = o;
  }
}

// Both bf16 packs of one conv from ONE read of the fp32 weight (Cin % 32 == Cout % 32 == 0).
// Block (co j0 .. j0+32, ci c*32 .. +32): the 32 contiguous 864-float runs w[co][c*32..][27]
// are converted to bf16 once into LDS (same rounding as pack_bf16x2), then both packs are
// written as 16-B pieces of the fragment-major layout (pack_bf16_off):
//   fwd   (c = ci/32, t, j = co, k = ci%32) = w[co][ci][t]
//   dgrad (c = co/32, t, j = ci, k = co%32) = w[co][ci][26 - t]
__global__ void __launch_bounds__(256) pack_conv3_bf16_both_kernel(const float* w, bf16_t* fwd, bf16_t* dgr,
                                                                   int Cout, int Cin) {
  __shared__ __attribute__((aligned(16))) uint16_t tb[32 * 864];
  const int chunk = blockIdx.y;
  const int j0 = blockIdx.x * 32;
  // all 27 loads of a thread in flight at once (the tile is 32 x 216 = 27 x 256 f32x4)
  f32x4_t v[27];
#pragma unroll
  for (int i = 0; i < 27; ++i) {
    const int e = threadIdx.x + i * 256, run = e / 216, q = e % 216;
    v[i] = __builtin_nontemporal_load(reinterpret_cast<const f32x4_t*>(w + ((long)(j0 + run) * Cin + chunk * 32) * 27) + q);
  }
#pragma unroll
  for (int i = 0; i < 27; ++i) {
    const int e = threadIdx.x + i * 256, run = e / 216, q = e % 216;
    uint2 o;
    o.x = pack_bf16x2(v[i][0], v[i][1]);
    o.y = pack_bf16x2(v[i][2], v[i][3]);
    *reinterpret_cast<uint2*>(tb + run * 864 + 4 * q) = o;
  }
  __syncthreads();
  for (int g = threadIdx.x; g < 27 * 128; g += 256) {
    const int t = g >> 7, co = (g >> 2) & 31, k8 = (g & 3) * 8;
    u32x4_t o;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      o[i] = (uint32_t)tb[co * 864 + (k8 + 2 * i) * 27 + t] | ((uint32_t)tb[co * 864 + (k8 + 2 * i + 1) * 27 + t] << 16);
    *reinterpret_cast<u32x4_t*>(fwd + pack_bf16_off(chunk, t, j0 + co, k8, Cout)) = o;
  }
  for (int g = threadIdx.x; g < 27 * 128; g += 256) {
    const int t = g >> 7, ci = (g >> 2) & 31, k8 = (g & 3) * 8, ts = 26 - t;
    u32x4_t o;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      o[i] = (uint32_t)tb[(k8 + 2 * i) * 864 + ci * 27 + ts] | ((uint32_t)tb[(k8 + 2 * i + 1) * 864 + ci * 27 + ts] << 16);
    *reinterpret_cast<u32x4_t*>(dgr + pack_bf16_off(j0 >> 5, t, chunk * 32 + ci, k8, Cin)) = o;
  }
}

// the pack16 forms of one 32 co x 32 ci tile from its bf16 copy in LDS (defined below pack16_off)
__device__ void pack16_tile_store(const uint16_t* tb, bf16_t* fwd16, bf16_t* dgr16, int j0, int ci0, int Cout,
                                  int Cin);

// Adam + the bf16 packs in one pass over the conv weights (the flat master is read once per
// step instead of once for Adam and once more for the packs).  One block per (conv, 32 co x
// 32 ci) tile of a table entry [off, Cout, Cin, fwd pack, dgrad pack, first tile, fwd16 pack,
// dgrad16 pack] (int64 each): the tile's 32 contiguous 864-float runs w[co][ci0..ci0+32][27]
// are updated in place (p, m, v, and g when scaled), the new weights converted to bf16 into
// LDS, and each non-null pack written: the general kernel's two as in
// pack_conv3_bf16_both_kernel, the 16x16x32 kernel's two as in pack16_conv3_kernel.
__global__ void __launch_bounds__(256) adam_pack_conv3_kernel(float* P, float* Gr, float* Mo, float* Vo,
                                                              const long long* tab, int ntab, AdamCoef c,
                                                              const float* gmul) {
  __shared__ __attribute__((aligned(16))) uint16_t tb[32 * 864];
  int ei = 0;
  while (ei + 1 < ntab && tab[8 * (ei + 1) + 5] <= (long long)blockIdx.x) ++ei;
  const long long* e = tab + 8 * ei;
  const long off = (long)e[0];
  const int Cout = (int)e[1], Cin = (int)e[2];
  bf16_t* fwd = reinterpret_cast<bf16_t*>(e[3]);
  bf16_t* dgr = reinterpret_cast<bf16_t*>(e[4]);
  bf16_t* fwd16 = reinterpret_cast<bf16_t*>(e[6]);
  bf16_t* dgr16 = reinterpret_cast<bf16_t*>(e[7]);
  const int local = blockIdx.x - (int)e[5];
  const int j0 = (local % (Cout / 32)) * 32, chunk = local / (Cout / 32);
  const float s = gmul ? c.gscale * gmul[0] : c.gscale;
  // ADAM_U iterations' four streams loaded before any is used: 4 x ADAM_U 16-B loads in flight
  // per thread (the stores of an iteration could alias the next one's loads for the compiler,
  // so without the explicit batch it keeps one iteration's loads in flight)
#ifndef ADAM_U
#define ADAM_U 3
#endif
  static_assert(27 % ADAM_U == 0, "ADAM_U divides the 27 iterations");
  for (int i0 = 0; i0 < 27; i0 += ADAM_U) {
    f32x4_t pv[ADAM_U], gv[ADAM_U], mv[ADAM_U], vv[ADAM_U];
    long idx[ADAM_U];
    int tbo[ADAM_U];
#pragma unroll
    for (int u = 0; u < ADAM_U; ++u) {
      const int q4 = threadIdx.x + (i0 + u) * 256, run = q4 / 216, q = q4 % 216;
      idx[u] = off + ((long)(j0 + run) * Cin + chunk * 32) * 27 + 4 * q;
      tbo[u] = run * 864 + 4 * q;
      // the fp32 master / gradient / moment streams (1.4 GB per step) bypass the caches
      pv[u] = __builtin_nontemporal_load(reinterpret_cast<const f32x4_t*>(P + idx[u]));
      gv[u] = __builtin_nontemporal_load(reinterpret_cast<const f32x4_t*>(Gr + idx[u]));
      mv[u] = __builtin_nontemporal_load(reinterpret_cast<const f32x4_t*>(Mo + idx[u]));
      vv[u] = __builtin_nontemporal_load(reinterpret_cast<const f32x4_t*>(Vo + idx[u]));
    }
#pragma unroll
    for (int u = 0; u < ADAM_U; ++u) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        float pk = pv[u][k], gk = gv[u][k], mk = mv[u][k], vk = vv[u][k];
        adam_update(pk, gk, mk, vk, c, s);
        pv[u][k] = pk; gv[u][k] = gk; mv[u][k] = mk; vv[u][k] = vk;
      }
      __builtin_nontemporal_store(pv[u], reinterpret_cast<f32x4_t*>(P + idx[u]));
      __builtin_nontemporal_store(mv[u], reinterpret_cast<f32x4_t*>(Mo + idx[u]));
      __builtin_nontemporal_store(vv[u], reinterpret_cast<f32x4_t*>(Vo + idx[u]));
      if (s != 1.f) __builtin_nontemporal_store(gv[u], reinterpret_cast<f32x4_t*>(Gr + idx[u]));
      uint2 o;
      o.x = pack_bf16x2(pv[u][0], pv[u][1]);
      o.y = pack_bf16x2(pv[u][2], pv[u][3]);
      *reinterpret_cast<uint2*>(tb + tbo[u]) = o;
    }
  }
  __syncthreads();
  if (fwd)
    for (int g = threadIdx.x; g < 27 * 128; g += 256) {
      const int t = g >> 7, co = (g >> 2) & 31, k8 = (g & 3) * 8;
      u32x4_t o;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        o[i] = (uint32_t)tb[co * 864 + (k8 + 2 * i) * 27 + t] | ((uint32_t)tb[co * 864 + (k8 + 2 * i + 1) * 27 + t] << 16);
      *reinterpret_cast<u32x4_t*>(fwd + pack_bf16_off(chunk, t, j0 + co, k8, Cout)) = o;
    }
  if (dgr)
    for (int g = threadIdx.x; g < 27 * 128; g += 256) {
      const int t = g >> 7, ci = (g >> 2) & 31, k8 = (g & 3) * 8, ts = 26 - t;
      u32x4_t o;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        o[i] = (uint32_t)tb[(k8 + 2 * i) * 864 + ci * 27 + ts] | ((uint32_t)tb[(k8 + 2 * i + 1) * 864 + ci * 27 + ts] << 16);
      *reinterpret_cast<u32x4_t*>(dgr + pack_bf16_off(j0 >> 5, t, chunk * 32 + ci, k8, Cin)) = o;
    }
  if (fwd16 || dgr16) pack16_tile_store(tb, fwd16, dgr16, j0, chunk * 32, Cout, Cin);
}

// fp32 build (bf16x6 packs): Adam + both three-part packs in one pass.  One block per (conv,
// 32 co x 16 ci) tile (the fp32 tile, 54 KiB, fits LDS where the 32 x 32 one would not): the
// 32 contiguous 432-float runs w[co][ci0..ci0+16][27] are updated in place as in
// adam_pack_conv3_kernel, the new fp32 weights kept in LDS, and each packed row -- 8 k
// values -> the B fragments [h|h] [m|h] [l|m] (split3x8, pack_conv3_kernel<x6_t>'s
// arithmetic) -- written as six 16-B stores:
//   fwd   [ci/8][t][co][48]   (k = ci)
//   dgrad [co/8][t][ci][48]   (k = co, tap mirrored)
__global__ void __launch_bounds__(256) adam_pack_conv3_x6_kernel(float* P, float* Gr, float* Mo, float* Vo,
                                                                 const long long* tab, int ntab, AdamCoef c,
                                                                 const float* gmul) {
  __shared__ float tf[32][16 * 27 + 1];  // [co][ci * 27 + t], rows padded by one float
  int ei = 0;
  while (ei + 1 < ntab && tab[8 * (ei + 1) + 5] <= (long long)blockIdx.x) ++ei;
  const long long* e = tab + 8 * ei;
  const long off = (long)e[0];
  const int Cout = (int)e[1], Cin = (int)e[2];
  bf16_t* fwd = reinterpret_cast<bf16_t*>(e[3]);
  bf16_t* dgr = reinterpret_cast<bf16_t*>(e[4]);
  const int local = blockIdx.x - (int)e[5];
  const int j0 = (local % (Cout / 32)) * 32, ci0 = (local / (Cout / 32)) * 16;
  const float s = gmul ? c.gscale * gmul[0] : c.gscale;
  // 32 runs of 108 f32x4 = 13.5 per thread: ADAM_X6_U iterations' four streams loaded before
  // any is used (adam_pack_conv3_kernel's batching; one iteration in flight per thread left
  // this kernel latency-bound at two 54-KiB blocks per CU)
#ifndef ADAM_X6_U
#define ADAM_X6_U 4
#endif
  for (int i0 = 0; i0 < 14; i0 += ADAM_X6_U) {
    f32x4_t pv[ADAM_X6_U], gv[ADAM_X6_U], mv[ADAM_X6_U], vv[ADAM_X6_U];
    long idx[ADAM_X6_U];
#pragma unroll
    for (int u = 0; u < ADAM_X6_U; ++u) {
      const int q4 = threadIdx.x + (i0 + u) * 256, run = q4 / 108, q = q4 % 108;
      idx[u] = off + ((long)(j0 + run) * Cin + ci0) * 27 + 4 * q;
      if (i0 + u < 14 && q4 < 32 * 108) {
        pv[u] = __builtin_nontemporal_load(reinterpret_cast<const f32x4_t*>(P + idx[u]));
        gv[u] = __builtin_nontemporal_load(reinterpret_cast<const f32x4_t*>(Gr + idx[u]));
        mv[u] = __builtin_nontemporal_load(reinterpret_cast<const f32x4_t*>(Mo + idx[u]));
        vv[u] = __builtin_nontemporal_load(reinterpret_cast<const f32x4_t*>(Vo + idx[u]));
      }
    }
#pragma unroll
    for (int u = 0; u < ADAM_X6_U; ++u) {
      const int q4 = threadIdx.x + (i0 + u) * 256, run = q4 / 108, q = q4 % 108;
      if (i0 + u >= 14 || q4 >= 32 * 108) break;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        float pk = pv[u][k], gk = gv[u][k], mk = mv[u][k], vk = vv[u][k];
        adam_update(pk, gk, mk, vk, c, s);
        pv[u][k] = pk; gv[u][k] = gk; mv[u][k] = mk; vv[u][k] = vk;
        tf[run][4 * q + k] = pk;
      }
      __builtin_nontemporal_store(pv[u], reinterpret_cast<f32x4_t*>(P + idx[u]));
      __builtin_nontemporal_store(mv[u], reinterpret_cast<f32x4_t*>(Mo + idx[u]));
      __builtin_nontemporal_store(vv[u], reinterpret_cast<f32x4_t*>(Vo + idx[u]));
      if (s != 1.f) __builtin_nontemporal_store(gv[u], reinterpret_cast<f32x4_t*>(Gr + idx[u]));
    }
  }
  __syncthreads();
  auto put = [](bf16_t* row, const float (&f)[8]) {
    u32x4_t h, m, l;
    split3x8(f, h, m, l);
    u32x4_t* o = reinterpret_cast<u32x4_t*>(row);
    o[0] = h; o[1] = h; o[2] = m; o[3] = h; o[4] = l; o[5] = m;
  };
  for (int r = threadIdx.x; r < 27 * 32 * 2; r += 256) {  // fwd rows (t, co, ci-chunk of 8)
    const int cc = r & 1, co = (r >> 1) & 31, t = r >> 6;
    float f[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) f[k] = tf[co][(cc * 8 + k) * 27 + t];
    put(fwd + ((((long)(ci0 / 8 + cc)) * 27 + t) * Cout + j0 + co) * 48, f);
  }
  for (int r = threadIdx.x; r < 27 * 16 * 4; r += 256) {  // dgrad rows (t, ci, co-chunk of 8)
    const int cc = r & 3, ci = (r >> 2) & 15, t = r >> 6;
    float f[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) f[k] = tf[cc * 8 + k][ci * 27 + 26 - t];
    put(dgr + ((((long)(j0 / 8 + cc)) * 27 + t) * Cin + ci0 + ci) * 48, f);
  }
}

// ------------------------------------------------------------------------------------
// Big-box forward / dgrad (bf16; the level-0/1 hot case: D % 8 == H % 8 == 0, W % 16 == 0,
// input channels in 16-channel chunks), PERSISTENT: one 8-wave workgroup per CU, one grid of
// at most #CU workgroups; workgroup (slot, cob) computes 8 x 8 x 16 = 1024-voxel boxes
// slot, slot + nslot, ... for its 64 output channels.  Wave w = (M-group mg = w & 3, N-tile
// nt = w >> 2) owns voxel rows [256 mg, 256 mg + 256) = 8 M-tiles and output channels
// [32 nt, 32 nt + 32), so every B fragment (weights, L2-resident; one contiguous 1 KiB load
// from the fragment-major pack, round 5) feeds 8 MFMAs and the two waves of a SIMD overlap
// one's operand waits with the other's MFMAs.
// The 10 x 10 x 18 halo of a chunk (32-B rows; the two 16-B halves swapped on odd row octets,
// so 16 consecutive rows hit 16 distinct bank groups) is double-buffered: the next chunk's
// halo -- the NEXT BOX's first chunk during a box's last chunk -- streams in by buffer
// LDS-DMA, one piece per thread and tap over the first 8 taps, and A fragments of tap t + 1
// are read while tap t's 8 MFMAs run; B loads run Dist taps ahead across chunk and box
// boundaries.  So only the first box of a workgroup waits for its operands; every later box
// starts on a landed halo.  Epilogue per box: + bias, bf16 channels staged through the
// M-group's 8 KiB LDS slice (two M-tiles at a time, the pair's channel halves) and
// written back as 16-B stores of whole 128-B channel rows (16 store instructions per wave and
// box, issued without waiting: the B waits of the next box's first taps count them).
// BatchNorm partials: per (M-group, channel) a running Chan merge over the boxes (count,
// mean, M2); one stats row per slot at the end.
// ------------------------------------------------------------------------------------
constexpr int kBgThreads = 512;  // 8 waves = 4 M-groups x 2 N-tiles, two waves per SIMD
constexpr int kBgHH = 10, kBgHW = 18;
constexpr int kBgBD = 8;                                                  // box depth
constexpr int kBgMT = 8;                                                  // M-tiles per wave
constexpr int kBgHalo = (kBgBD + 2) * kBgHH * kBgHW;                      // rows x 32 B
constexpr int kBgPieces = (2 * kBgHalo + kBgThreads - 1) / kBgThreads;    // DMA pieces / thread (8)
// pieces pc = tid + 512 j; the last round (j = 7) holds real rows only for wave 0: the other
// waves aim it at a 1 KiB dummy slot (out-of-range source: no memory traffic) so every wave
// issues the same count; a buffer holds rows up to wave 0's last piece
constexpr int kBgBuf = ((kBgPieces - 1) * kBgThreads + 64) * 16;
constexpr int kBgDummy = 1024;
constexpr int kBgStage = 64 * 128;                                        // per-M-group store slice
constexpr int kBgRed = 4 * 64 * 3 * 4;                                    // BN moments
constexpr int kBgLds = 2 * kBgBuf + kBgDummy + 4 * kBgStage + kBgRed + 64 * 4;  // + bias
// BNIN: the input BatchNorm's scale / shift table [2][kBgBnMax] floats after that
constexpr int kBgBnMax = 128;
constexpr int kBgBnOff = kBgLds;
constexpr int kBgLdsBn = kBgLds + 2 * kBgBnMax * 4;
#ifndef BG_DIST
#define BG_DIST 8  // 2: 1-1.5 % slower big-box launches (A/B, profiles/r4_bg_dist_ab.txt)
#endif
// ablation builds only (tests/tools/big_abl.py; 0 in the product): 1 halo DMA reads nothing
// (out-of-range source, the same instructions), 2 no output stores, 4 no MFMAs (operands still
// read), 8 no weight loads after the prologue, 16 no A-fragment LDS reads
#ifndef BG_ABL
#define BG_ABL 0
#endif
constexpr int kBgDist = BG_DIST;           // B prefetch distance (taps); (Dist + 1) | 27
constexpr int kBgEpiStores = kBgMT * 2;    // 16-B stores per wave and box
static_assert(27 % (kBgDist + 1) == 0, "B ring index must continue across chunks");
static_assert(kBgLdsBn <= 160 * 1024, "LDS");

// hidden 16-B global load (the compiler's waitcnt pass does not count it): retired by
// vm_wait2<N>, which also orders the register's readers after the wait
__device__ __forceinline__ void gload16(s16x8_t& dst, const void* ptr) {
  asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(dst) : "v"(ptr) : "memory");
}
// the same through a buffer descriptor (bounds-checked: out of range reads zeros), one VGPR
// byte offset per address, immediate offset Imm
template <int Imm> __device__ __forceinline__ void bload16(s16x8_t& dst, i32x4_t rsrc, uint32_t voff) {
  asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen offset:%3" : "=v"(dst) : "v"(voff), "s"(rsrc), "n"(Imm)
               : "memory");
}
template <int N> __device__ __forceinline__ void vm_wait1(s16x8_t& a) {
  static_assert(N >= 0 && N <= 63, "vmcnt");
  asm volatile("s_waitcnt vmcnt(%1)" : "+v"(a) : "n"(N) : "memory");
}
// vector-memory ops issued after B(t)'s load by the time tap t waits for it: every tap s
// issues B(s + D) then piece(s) (s < P, chunk-relative, every chunk alike)
template <int P> constexpr int bg_piece(int s) { return ((s % 27) + 27) % 27 < P ? 1 : 0; }
template <int P, int Dist> constexpr int bg_wait(int t) {
  int n = bg_piece<P>(t - Dist);
  for (int s = t - Dist + 1; s <= t; ++s) n += 1 + bg_piece<P>(s);
  return n;
}
template <int N> __device__ __forceinline__ void vm_wait() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

// BNIN (pcms_conv3_fwd_bnin, single-source inputs of <= kBgBnMax channels): the input is
// relu(x * isc + ish) -- the previous BatchNorm + ReLU applied in the staging path instead of
// a separate HBM pass.  At a chunk's end each thread rewrites the pieces it staged for the
// next chunk in LDS (their DMA has landed by the chunk-end vmcnt wait; out-of-range pieces,
// the zero padding, are left zero), before the barrier that publishes the buffer.
template <bool BNIN = false>
__global__ void __launch_bounds__(kBgThreads, 1) conv3_fwd_big_kernel(Conv3Params p, uint32_t x0bytes,
                                                                     uint32_t x1bytes) {
  constexpr int MT = kBgMT;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // wave = (M-group mg: box voxel rows 256 mg ..; N-tile nt: output channels 32 nt .. 32 nt + 31)
  const int mg = wave & 3, nt = wave >> 2;
  const int Cout = p.Cout, ncob = Cout >> 6;
  // logical workgroup id: consecutive ids on one XCD (dispatch is round-robin over 8), output
  // channel block fastest, so the workgroups sharing a halo (and neighbouring boxes) share L2
  const int G = gridDim.x;
  const int lg = (G & 7) == 0 ? (blockIdx.x & 7) * (G >> 3) + (blockIdx.x >> 3) : blockIdx.x;
  const int cob = lg % ncob, slot = lg / ncob, nslot = G / ncob;
  const int nbox = p.N * p.nbd * p.nbh * p.nbw;
  // box walk: slot, slot + nslot, ... (a d-column walk and sc1 / nt output stores measured
  // no different, profiles/r5_big_walk_storepolicy_ab.txt)
  const int box_step = nslot, box_end = nbox, box0 = slot;
  const int co_base = cob * 64;
  auto origin = [&](int box, int& n, int& d0, int& h0, int& w0) {
    int q = box;
    const int bwi = q % p.nbw; q /= p.nbw;
    const int bhi = q % p.nbh; q /= p.nbh;
    const int bdi = q % p.nbd;
    n = q / p.nbd;
    d0 = bdi * kBgBD; h0 = bhi * 8; w0 = bwi * 16;
  };

  const i32x4_t xr0 = buffer_desc(p.x0, x0bytes);
  const i32x4_t xr1 = buffer_desc(p.x1 ? p.x1 : p.x0, x1bytes);
  const uint32_t lds0 = lds_addr(lds);
  // live = false (past the last box): the piece is still issued (the vmcnt arithmetic is the
  // same for every chunk) but reads out of range = zeros into the idle buffer
  auto stage_piece = [&](int n, int d0, int h0, int w0, int chunk, int buf, int j, bool live) {
    const int c = chunk * 16;
    const bool first = c < p.c0;  // workgroup-uniform: the chunk lies in x0 or in x1
    const uint32_t stride = first ? p.c0 : p.c1;
    const uint32_t cofs = first ? c : c - p.c0;
    // piece j of this thread: halo row hv = pc / 2, logical 16-B half (pc & 1) swapped on odd
    // row octets (recomputed per chunk: a few VALU against 432 MFMAs, no registers held)
    const int pc = opaque(tid) + j * kBgThreads;
    const int hv = pc >> 1;
    const int hw_ = hv % kBgHW, t_ = hv / kBgHW, hh_ = t_ % kBgHH, hd_ = t_ / kBgHH;
    const int gd = d0 + hd_ - 1, gh = h0 + hh_ - 1, gw = w0 + hw_ - 1;
    uint32_t voff = kOOB;
    if (live && hv < kBgHalo && (unsigned)gd < (unsigned)p.D && (unsigned)gh < (unsigned)p.H &&
        (unsigned)gw < (unsigned)p.W && !(BG_ABL & 1))
      voff = ((uint32_t)(((n * p.D + gd) * p.H + gh) * p.W + gw) * stride + cofs +
              (uint32_t)((pc & 1) ^ ((hw_ >> 3) & 1)) * 8u) * 2u;
    const bool dummy = j == kBgPieces - 1 && wave > 0;  // wave-uniform
    const uint32_t lb = __builtin_amdgcn_readfirstlane(
        dummy ? lds0 + 2 * kBgBuf : lds0 + buf * kBgBuf + (wave * 64 + j * kBgThreads) * 16);
    dma16(first ? xr0 : xr1, lb, dummy ? kOOB : voff, 0);
    // BNIN: bit j = a real piece; bit 8 + j = its logical channel half
    return (!dummy && voff != kOOB ? 1u << j : 0u) | ((uint32_t)((pc & 1) ^ ((hw_ >> 3) & 1)) << (8 + j));
  };
  // BNIN: the staged pieces of buffer `buf` (chunk `chunk`) -> relu(x sc + sh) in place
  float* bnt = reinterpret_cast<float*>(lds + kBgBnOff);  // reserved by kBgLdsBn (BNIN launches)
  auto bn_apply = [&](int buf, int chunk, uint32_t pm) {
#pragma unroll
    for (int j = 0; j < kBgPieces; ++j) {
      if (!((pm >> j) & 1)) continue;
      const int pc = tid + j * kBgThreads;
      u32x4_t* q = reinterpret_cast<u32x4_t*>(lds + buf * kBgBuf + pc * 16);
      const int c = chunk * 16 + ((pm >> (8 + j)) & 1) * 8;
      const f32x4_t s0 = *reinterpret_cast<const f32x4_t*>(bnt + c), s1 = *reinterpret_cast<const f32x4_t*>(bnt + c + 4);
      const f32x4_t h0 = *reinterpret_cast<const f32x4_t*>(bnt + kBgBnMax + c);
      const f32x4_t h1 = *reinterpret_cast<const f32x4_t*>(bnt + kBgBnMax + c + 4);
      const float sc[8] = {s0[0], s0[1], s0[2], s0[3], s1[0], s1[1], s1[2], s1[3]};
      const float sh[8] = {h0[0], h0[1], h0[2], h0[3], h1[0], h1[1], h1[2], h1[3]};
      u32x4_t v = *q;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        v[i] = pack_bf16x2(bn_relu1(__uint_as_float(v[i] << 16), sc[2 * i], sh[2 * i]),
                           bn_relu1(__uint_as_float(v[i] & 0xffff0000u), sc[2 * i + 1], sh[2 * i + 1]));
      *q = v;
    }
  };
  if constexpr (BNIN) {
    if (tid < p.Cin) { bnt[tid] = p.isc[tid]; bnt[kBgBnMax + tid] = p.ish[tid]; }
    __syncthreads();
  }

  // A fragment byte offsets in a halo buffer: MFMA row r = 256 wave + 32 mt + perm32(lane)
  // is box voxel (2 wave + mt / 4, 2 (mt % 4) + prow / 16, prow % 16).  The half swizzle
  // depends on the halo w coordinate only, so for each kw the (kd, kh) part of a tap is a
  // constant row offset (kd * 10 + kh) * 18 * 32 bytes folded into the ds_read immediate.
  // One base register per kw (recomputed per chunk); the M-tile and (kd, kh) parts are
  // ds_read immediates.
  // B fragments (weights, packed [Cin/32][27][Cout][32]; 16-channel chunk c = half c & 1 of
  // 32-chunk c >> 1) come through hidden loads Dist taps ahead: vector-memory returns are
  // in order, so a wait on B(t) also retires every halo piece issued before it; the pieces
  // get >= Dist taps to arrive from HBM before anything waits on them.
  // B address: (chunk, tap) byte offset (uniform) + one per-lane byte offset, through a
  // descriptor over the whole pack
  const int nchunk = p.Cin >> 4;
  const uint32_t tap_bytes = (uint32_t)Cout * 64u;
  const i32x4_t wr = buffer_desc(p.w, (uint32_t)(p.Cin >> 5) * 27u * tap_bytes);
  bool bl_prologue = true;  // BG_ABL & 8: only the prologue's weight loads run
  auto load_b = [&](s16x8_t& dst, int chunk, int tap, uint32_t boff) {
    if ((BG_ABL & 8) && !bl_prologue) return;
    // fragment-major pack (pack_bf16_off): the (32-chunk, tap) rows, boff = this wave's row
    // tile and lane, then the k-step (chunk & 1): one contiguous 1 KiB per wave
    const uint32_t off = boff + (uint32_t)((chunk >> 1) * 27 + tap) * tap_bytes + (uint32_t)(chunk & 1) * 1024u;
    bload16<0>(dst, wr, off);
  };

  // epilogue constants: column j of N-tile nt = channel 32 nt + j; two-pointer output split at
  // cy0 (workgroup-uniform)
  // (bias and the running BatchNorm moments live in LDS between boxes, not in registers)
  float* red = reinterpret_cast<float*>(lds + 2 * kBgBuf + kBgDummy + 4 * kBgStage);  // [mg][64][3]
  float* bls = red + 4 * 64 * 3;                                           // [64]
  if (tid < 64) bls[tid] = p.bias ? p.bias[co_base + tid] : 0.f;
  const bool to0 = co_base < p.cy0;
  const long ys = to0 ? p.cy0 : Cout - p.cy0;
  const int yc0 = to0 ? co_base : co_base - p.cy0;
  // output through a descriptor too (stores out of range are dropped; the host checks
  // every byte offset fits 31 bits)
  const __amdgpu_buffer_rsrc_t yr = __builtin_amdgcn_make_buffer_rsrc(
      to0 ? p.y0 : p.y1, (short)0, (int)(p.nvox * ys * 2), 0x00020000);
  char* stg = lds + 2 * kBgBuf + kBgDummy + mg * kBgStage;  // shared by the M-group's two waves
  int nbdone = 0;  // boxes merged into the running moments (uniform: kept in an SGPR)

  f32x16_t acc[MT];
  s16x8_t bset[kBgDist + 1];
  int box = box0;
  int n, d0, h0, w0;
  origin(box, n, d0, h0, w0);
  // Short boxes (4 chunks): every CU would reach its box boundary -- the vmcnt(0), the 128 KiB
  // store burst and the next halo's first pieces -- at the same moment; starting slot s
  // (s % 4) x ~16k cycles late spreads those bursts (measured 517 -> 433 us at level 0,
  // 64 -> 64; no effect with 8+ chunks, so not applied there).
  if (nchunk <= 4)
    for (int i = 0; i < 2 * (slot & 3); ++i) __builtin_amdgcn_s_sleep(127);
  uint32_t pmask = 0;  // BNIN: the pieces staged for the next chunk (stage_piece bits)
#pragma unroll
  for (int j = 0; j < kBgPieces; ++j) pmask |= stage_piece(n, d0, h0, w0, 0, 0, j, true);
#pragma unroll
  for (int t = 0; t < kBgDist; ++t) load_b(bset[t], 0, t, (uint32_t)(((co_base >> 5) + nt) * 2048 + lane * 16));
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  bl_prologue = false;
  if constexpr (BNIN) bn_apply(0, 0, pmask);
  __syncthreads();
  int buf = 0;
  while (true) {
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][e] = 0.f;
    const int nbx = box + box_step;
    const bool has_next = nbx < box_end;
    int nn = n, nd0 = d0, nh0 = h0, nw0 = w0;
    if (has_next) origin(nbx, nn, nd0, nh0, nw0);
    // one chunk: 27 taps.  Chunk 0 (peeled, Slack): B(t < Dist) were issued before the
    // previous box's 32 epilogue stores, so those waits count them as well; in a workgroup's
    // first box the prologue's vmcnt(0) already retired B(t < Dist), the looser count is safe.
    auto run_chunk = [&](int chunk, auto slack_tag) {
      constexpr bool Slack = decltype(slack_tag)::value;
      const bool last = chunk + 1 == nchunk;
      const bool live = !last || has_next;
      const int sn = last ? nn : n, sd = last ? nd0 : d0, sh = last ? nh0 : h0, sw = last ? nw0 : w0;
      const int schunk = last ? 0 : chunk + 1;
      const char* hl = lds + buf * kBgBuf;
      const int lo = opaque(lane);
      const int prow = perm32(lo & 31), hs = lo >> 5;
      const int hbase = ((2 * mg * kBgHH + (prow >> 4)) * kBgHW + (prow & 15)) * 32;
      int swk[3];
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) swk[kw] = hbase + kw * 32 + ((hs ^ ((((prow & 15) + kw) >> 3) & 1)) << 4);
      const uint32_t boff = (uint32_t)(((co_base >> 5) + nt) * 2048 + lo * 16);
      auto read_a1 = [&](int tap, int mt) {
        if constexpr ((BG_ABL & 16) != 0) tap = 0;
        const int kd = tap / 9, kh = (tap / 3) % 3, kw = tap % 3;
        return *reinterpret_cast<const s16x8_t*>(hl + swk[kw] + (kd * kBgHH + kh) * kBgHW * 32 +
                                                 ((mt >> 2) * kBgHH + 2 * (mt & 3)) * kBgHW * 32);
      };
      // A fragments roll through one register set: right after M-tile mt's two MFMAs of tap t
      // its fragment of tap t + 1 is read (14 MFMAs of slack before its first use)
      s16x8_t a[MT];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) a[mt] = read_a1(0, mt);
      // per tap: B(tap + D) (the set index runs on across chunks: (D + 1) | 27), one halo
      // piece of the next chunk (taps < 15); wait for B(tap); 16 MFMAs
      static_for<27>([&](auto tc) {
        constexpr int tap = decltype(tc)::value;
        constexpr int tn = tap + kBgDist;
        if constexpr (tn < 27) load_b(bset[tn % (kBgDist + 1)], chunk, tn, boff);
        else load_b(bset[tn % (kBgDist + 1)], schunk, tn - 27, boff);
        if constexpr (tap < kBgPieces) {
          const uint32_t bits = stage_piece(sn, sd, sh, sw, schunk, buf ^ 1, tap, live);
          if constexpr (BNIN) pmask = (tap == 0 ? 0u : pmask) | bits;
        }
        s16x8_t& b = bset[tap % (kBgDist + 1)];
        constexpr int extra = (Slack && tap < kBgDist) ? kBgEpiStores : 0;
        vm_wait1<bg_wait<kBgPieces, kBgDist>(tap) + extra>(b);
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
          if constexpr ((BG_ABL & 4) != 0) asm volatile("" ::"v"(a[mt]), "v"(b));
          else acc[mt] = mfma(a[mt], b, acc[mt]);
          if constexpr (tap + 1 < 27 && (BG_ABL & 16) == 0) a[mt] = read_a1(tap + 1, mt);
        }
      });
      // the next chunk's halo has landed (the newest piece is followed by the B loads of the
      // remaining taps) and every wave is done with buf.  After a box's last chunk retire
      // everything: the epilogue needs registers, and the compiler may move (or, after the
      // workgroup's last box, reuse) the destinations of the next box's B loads -- they
      // must hold landed data by then (costs one L2 round trip per box).
      if (!last) vm_wait<27 - kBgPieces>();
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if constexpr (BNIN) bn_apply(buf ^ 1, schunk, pmask);
      __syncthreads();
      buf ^= 1;
    };
    run_chunk(0, std::true_type{});
    for (int chunk = 1; chunk < nchunk; ++chunk) run_chunk(chunk, std::false_type{});

    // ---- epilogue of this box, two M-tiles at a time: + bias, bf16 channels into the
    // M-group's LDS slice (row = 32 mm + C row, 128 B of 64 channels; the two waves of the
    // group write channels 0-31 / 32-63), read back as 4 x 16 B per lane and wave = whole
    // 128-B channel rows, 16-B stores.  BatchNorm moments in the same pass, shifted by K
    // (the running mean; the bias before the first box): box mean K + S1 / n, M2 = S2 -
    // S1^2 / n, Chan-merged into the running moments.
    // (lane-dependent offsets from an opaque lane copy: box-invariant, the compiler would
    // hoist them out of the box loop and spill them)
    const int lane_o = opaque(lane);
    const long plane = (long)p.H * p.W;
    const long vbase = (((long)n * p.D + d0) * p.H + h0) * p.W + w0;
    char* wst = stg + (lane_o & 31) * 2 + nt * 64 + (lane_o >> 5) * 512;
    float* rme = red + (mg * 64 + 32 * nt + (lane_o & 31)) * 3;  // [ch][mean, M2, n] of this wave's channel
    const float bias0 = bls[32 * nt + (lane_o & 31)];
    const bool relu = p.accumulate & PCMS_CONV_RELU;  // eval: BatchNorm folded (no stats then)
    const float rn = (float)nbdone * (32.f * MT);
    const float K0 = nbdone ? rme[0] : bias0;
    const float c0s = bias0 - K0;  // d = acc + bias - K
    float S1 = 0.f, S2 = 0.f;
#pragma unroll
    for (int pass = 0; pass < MT / 2; ++pass) {
#pragma unroll
      for (int mm = 0; mm < 2; ++mm)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int row = mm * 32 + (e & 3) + 8 * (e >> 2);
          const float v0 = acc[2 * pass + mm][e];
          *reinterpret_cast<bf16_t*>(wst + row * 128) = f2bf(relu ? fmaxf(v0 + bias0, 0.f) : v0 + bias0);
          const float e0 = v0 + c0s;
          S1 += e0;
          S2 = fmaf(e0, e0, S2);
        }
      // both waves of the M-group have written their channels of the slice (raw barrier:
      // __syncthreads() would also drain this wave's stores of the previous pass)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int row = (4 * nt + k) * 8 + (lane_o >> 3), c16 = lane_o & 7;
        const u32x4_t v = *reinterpret_cast<const u32x4_t*>(stg + row * 128 + c16 * 16);
        const int mt = 2 * pass + (row >> 5), pr = perm32(row & 31);
        const int rd = 2 * mg + (mt >> 2), rh = 2 * (mt & 3) + (pr >> 4), rw = pr & 15;
        const long vox = vbase + (long)rd * plane + (long)rh * p.W + rw;
        if constexpr ((BG_ABL & 2) == 0)
          __builtin_amdgcn_raw_buffer_store_b128(v, yr, (int)((vox * ys + yc0 + c16 * 8) * 2), 0, 0);
        else
          asm volatile("" ::"v"(v), "v"((int)vox));
      }
      // both waves are done reading the slice before the next pass rewrites it
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
    {
      constexpr float nb = 32.f * MT;  // voxels per wave and box
      const float nnew = rn + nb;
      const float s1 = S1 + __shfl_xor(S1, 32, 64);
      const float s2 = S2 + __shfl_xor(S2, 32, 64);
      const float mbox = K0 + s1 / nb;
      const float m2b = fmaxf(s2 - s1 * s1 / nb, 0.f);
      const float rmean = nbdone ? rme[0] : 0.f, rm2 = nbdone ? rme[1] : 0.f;
      const float delta = mbox - rmean;
      if ((lane_o >> 5) == 0) {
        rme[0] = rmean + delta * (nb / nnew);
        rme[1] = rm2 + m2b + delta * delta * (rn * nb / nnew);
        rme[2] = nnew;
      }
      ++nbdone;
    }
    if (!has_next) break;
    box = nbx;
    n = nn; d0 = nd0; h0 = nh0; w0 = nw0;
  }

  if (!p.stats) return;
  // one stats row per slot: Chan merge of the 4 waves' running moments (mean, M2, n)
  __syncthreads();
  if (tid < 64) {
    float S = 0.f, Nn = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      S += red[(w * 64 + tid) * 3] * red[(w * 64 + tid) * 3 + 2];
      Nn += red[(w * 64 + tid) * 3 + 2];
    }
    const float m = S / Nn;
    float M2 = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const float c = red[(w * 64 + tid) * 3 + 2];
      const float d = red[(w * 64 + tid) * 3] - m;
      M2 += red[(w * 64 + tid) * 3 + 1] + c * d * d;
    }
    float* st = p.stats + ((long)slot * Cout + co_base + tid) * 2;
    st[0] = S;
    st[1] = M2;
    if (tid == 0 && cob == 0) p.stats[(long)nslot * Cout * 2 + slot] = Nn;
  }
}


// ------------------------------------------------------------------------------------
// Big-box forward / dgrad on v_mfma_f32_16x16x32_bf16 (round 5; pcms_conv3_fwd16).  The same
// persistent 8-wave workgroup, 8 x 8 x 16 boxes, 16-channel chunks and LDS-DMA halo pipeline
// as conv3_fwd_big_kernel, with the MFMA shape changed: K = 32 = a PAIR of taps x 16 channels
// (lanes 0-31 of a fragment hold tap 2 s, lanes 32-63 tap 2 s + 1; 14 k-steps per chunk, the
// 28th tap a zero weight), wave w = box d-plane w: 8 M-tiles (its 8 h-rows of 16 voxels) x 4
// N-tiles (all 64 output channels), so per k-step 8 A reads + 4 B loads feed 32 MFMAs -- half
// the A bytes per FLOP of the 32x32x16 kernel.  Why: the big-box convs run power-capped
// (1.4-1.9 GHz in step, profiles/r5_layer_times_clock.json), and this inner loop does the same
// FLOPs for ~11 % less time on every CU at once (tests/kexp/mfma_shape.hip:
// profiles/r5_mfma_shape_probe.txt: 1505-1529 vs 1358-1370 TFLOP/s, at 2.00-2.06 vs 1.90-1.94
// GHz).  Halo rows stay 32 B (16 channels) without a swizzle: a 16-lane ds_read_b128 group reads
// rows {0-3, 12-15} of one half and {4-11} of the other, all 64 banks once.  B fragments come
// from the pack16 layout (pack16_off: one contiguous 1 KiB per (chunk, tap pair, 16-channel
// tile)).  Epilogue: each wave stages one M-tile at a time (16 voxels x 64 channels, 144-B rows)
// in its own LDS slice -- no cross-wave barrier -- and writes whole 128-B channel rows.
// ------------------------------------------------------------------------------------
constexpr int kB6Steps = 14;                       // tap pairs per chunk
// B prefetch distance (k-steps; (Dist + 1) | 14 so the ring index continues across chunks): 1
// with two waves per SIMD (8-deep boxes), 6 with one (4-deep: the other wave no longer covers
// a weight fetch that misses L2)
#ifndef B6_DIST4
#define B6_DIST4 6  // (A/B builds: -DB6_DIST4=1)
#endif
// NT = 8 (128 output channels per wave, 256 accumulators: one wave per SIMD only) keeps two
// register sets, Dist 1
template <int BD, int NT = 4> constexpr int b6_dist() { return BD == 8 || NT == 8 ? 1 : B6_DIST4; }
// geometry of a box of BD d-planes (one wave each): 8 (levels 0-1) or 4 (level 2, whose 8-deep
// boxes would leave half the CUs idle; and, with NT = 8 N-tiles per wave, the 128-channel
// blocks of levels 0-1: one staged halo feeds twice the MFMAs).  pieces pc = tid + T j; the
// wave-instructions wholly past the halo's 2 Halo pieces aim at a 1 KiB dummy slot
// (out-of-range source: no memory traffic) so every wave issues the same count; a buffer
// holds rows up to the last real piece.  Epilogue slice rows: NT x 16 channels bf16 + 16 B
// (conflict-free 2-B writes), 16 rows (one M-tile) per wave.
template <int BD, int NT = 4> struct B6G {
  static constexpr int T = BD * 64;
  static constexpr int CO = NT * 16;                                    // channels per workgroup
  static constexpr int Halo = (BD + 2) * kBgHH * kBgHW;                 // rows x 32 B
  static constexpr int Pieces = (2 * Halo + T - 1) / T;                 // DMA pieces / thread
  static constexpr int Buf = (2 * Halo + 63) / 64 * 1024;
  static constexpr int Row = CO * 2 + 16;
  static constexpr int Slice = 16 * Row;
  static constexpr int EpiStores = 8 * NT / 2;                          // 16-B stores per wave and box
  static constexpr int SliceOff = 2 * Buf + kBgDummy;
  static constexpr int RedOff = SliceOff + BD * Slice;
  static constexpr int Lds = RedOff + BD * CO * 3 * 4 + CO * 4;         // + bias
  static constexpr int BnOff = Lds;
  static constexpr int LdsBn = Lds + 2 * kBgBnMax * 4;
  // split-K form (fp32 partial rows): its own slice of 16 rows x CO fp32 (+ 16 B) per wave
  static constexpr int Row32 = CO * 4 + 16;
  static constexpr int LdsSplit = SliceOff + BD * 16 * Row32;
  static constexpr int EpiStores32 = 8 * CO / 16;                       // 16-B stores per wave and box
  static_assert(LdsSplit <= 160 * 1024, "LDS");
  static_assert(Pieces <= kB6Steps, "one piece per k-step");
  static_assert((Pieces - 2) * T + (BD - 1) * 64 < 2 * Halo, "dummy pieces in the last round only");
  static_assert(LdsBn <= 160 * 1024, "LDS");
};
static_assert(B6G<8>::Buf == kBgBuf && B6G<8>::Pieces == kBgPieces, "8-deep geometry");
static_assert(B6G<8>::Row == 144 && B6G<8>::EpiStores == 16, "64-channel slice rows");

// box w width WB: 16 (levels 0-2: an M-tile is one h-row of 16 w) or 8 (level 3: an M-tile is
// two h-rows of 8 w); the box is BD d-planes x (128 / WB) h x WB w, its halo plane HH x HW
// rows (10 x 18 or 18 x 10: 180 rows either way)
template <int WB> struct B6W {
  static constexpr int BH = 128 / WB, HH = BH + 2, HW = WB + 2;
  static constexpr int MTR = (16 / WB) * HW;  // halo rows between M-tiles
};
static_assert(B6W<16>::HH == kBgHH && B6W<16>::HW == kBgHW && B6W<8>::HH * B6W<8>::HW == kBgHH * kBgHW, "halo");
// halo row offset of tap t; the zero-weight 28th tap reads tap 26's rows
template <int WB = 16> __host__ __device__ constexpr int b6_tapoff(int t) {
  return t > 26 ? b6_tapoff<WB>(26) : ((t / 9) * B6W<WB>::HH + (t / 3) % 3) * B6W<WB>::HW + t % 3;
}
// retire the hidden loads of the B fragments of a step (and everything issued before)
template <int N> __device__ __forceinline__ void vm_wait4(s16x8_t (&b)[4]) {
  static_assert(N >= 0 && N <= 63, "vmcnt");
  asm volatile("s_waitcnt vmcnt(%4)" : "+v"(b[0]), "+v"(b[1]), "+v"(b[2]), "+v"(b[3]) : "n"(N) : "memory");
}
template <int N> __device__ __forceinline__ void vm_wait4(s16x8_t (&b)[8]) {
  static_assert(N >= 0 && N <= 63, "vmcnt");
  asm volatile("s_waitcnt vmcnt(%8)"
               : "+v"(b[0]), "+v"(b[1]), "+v"(b[2]), "+v"(b[3]), "+v"(b[4]), "+v"(b[5]), "+v"(b[6]), "+v"(b[7])
               : "n"(N) : "memory");
}
template <int P> constexpr int b6_piece(int s) { return ((s % kB6Steps) + kB6Steps) % kB6Steps < P ? 1 : 0; }
// vector-memory ops issued after the last of B(t)'s NT loads by the time step t waits for it:
// every step u issues B(u + D) (NT loads) then piece(u) (u < P)
template <int P, int Dist, int NT = 4> constexpr int b6_wait(int t) {
  int n = b6_piece<P>(t - Dist);
  for (int u = t - Dist + 1; u <= t; ++u) n += NT + b6_piece<P>(u);
  return n;
}

// WB: box w width (B6W).  SPLIT (level 3): the workgroups of a (slot, co block) cover 1 / nsplit of
// the input chunks each (p.chunks_per_split) and write fp32 partial rows p.yacc[split][vox][co]
// (no bias / statistics: pcms_split_epilogue sums the splits in a fixed order)
template <bool BNIN = false, int BD = 8, int NT = 4, int WB = 16, bool SPLIT = false>
__global__ void __launch_bounds__(BD * 64, 1) conv3_fwd_b16_kernel(Conv3Params p, uint32_t x0bytes,
                                                                  uint32_t x1bytes) {
  typedef B6G<BD, NT> G6;
  typedef B6W<WB> GW;
  static_assert(NT == 4 || (NT == 8 && BD == 4), "128-channel blocks: one wave per SIMD");
  static_assert(!SPLIT || (!BNIN && NT == 4), "split-K form: plain 64-channel blocks");
  constexpr int CO = G6::CO;
  // kT (64-channel blocks): the MFMA runs weights x activations, so a lane's accumulator holds
  // 4 consecutive output channels of one voxel (channel-major D) -- the epilogue stores them
  // straight from registers (8 B of bf16, or 16 B of fp32 partial rows) instead of transposing
  // through the LDS slice
  constexpr bool kT = NT == 4;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
#if PCMS_SETPRIO & 2
  if (BD == 8 && wave >= 4) __builtin_amdgcn_s_setprio(1);  // the younger wave of each SIMD pair
#endif
  const int Cout = p.Cout, ncob = Cout / CO;
  const int G = gridDim.x;
  const int lg = (G & 7) == 0 ? (blockIdx.x & 7) * (G >> 3) + (blockIdx.x >> 3) : blockIdx.x;
  const int nsplit = SPLIT ? p.nchunk / p.chunks_per_split : 1;
  const int cob = lg % ncob, split = SPLIT ? (lg / ncob) % nsplit : 0;
  const int slot = lg / ncob / nsplit, nslot = G / ncob / nsplit;
  const int nbox = p.N * p.nbd * p.nbh * p.nbw;
  const int co_base = cob * CO;
  auto origin = [&](int box, int& n, int& d0, int& h0, int& w0) {
    int q = box;
    const int bwi = q % p.nbw; q /= p.nbw;
    const int bhi = q % p.nbh; q /= p.nbh;
    const int bdi = q % p.nbd;
    n = q / p.nbd;
    d0 = bdi * BD; h0 = bhi * GW::BH; w0 = bwi * WB;
  };
  const i32x4_t xr0 = buffer_desc(p.x0, x0bytes);
  const i32x4_t xr1 = buffer_desc(p.x1 ? p.x1 : p.x0, x1bytes);
  const uint32_t lds0 = lds_addr(lds);
  // halo piece j of this thread: row pc / 2 (32 B), 16-B half pc & 1 (channels 8 half ..),
  // no swizzle; live = false: still issued (the vmcnt arithmetic), reads out of range = zeros.
  // The piece's voxel (pvox, -1 outside the volume) depends on the box only: formed when a
  // box's first chunk is staged (fresh) and reused for its other chunks (one multiply-add then);
  // 4-deep boxes only (one wave per SIMD: registers to spare; the 8-deep kernel spills with it)
  constexpr bool kCache = BD == 4;
  int pvox[kCache ? G6::Pieces : 1];
  auto stage_piece = [&](int n, int d0, int h0, int w0, int chunk, int buf, int j, bool live, bool fresh) {
    const int c = chunk * 16;
    const bool first = c < p.c0;
    const uint32_t stride = first ? p.c0 : p.c1;
    const uint32_t cofs = first ? c : c - p.c0;
    const int pc = opaque(tid) + j * G6::T;
    uint32_t voff = kOOB;
    if constexpr (kCache) {
      if (fresh) {
        const int hv = pc >> 1;
        const int hw_ = hv % GW::HW, t_ = hv / GW::HW, hh_ = t_ % GW::HH, hd_ = t_ / GW::HH;
        const int gd = d0 + hd_ - 1, gh = h0 + hh_ - 1, gw = w0 + hw_ - 1;
        pvox[j] = (hv < G6::Halo && (unsigned)gd < (unsigned)p.D && (unsigned)gh < (unsigned)p.H &&
                   (unsigned)gw < (unsigned)p.W) ? ((n * p.D + gd) * p.H + gh) * p.W + gw : -1;
      }
      if (live && pvox[j] >= 0) voff = ((uint32_t)pvox[j] * stride + cofs + (uint32_t)(pc & 1) * 8u) * 2u;
    } else {
      (void)fresh;
      const int hv = pc >> 1;
      const int hw_ = hv % GW::HW, t_ = hv / GW::HW, hh_ = t_ % GW::HH, hd_ = t_ / GW::HH;
      const int gd = d0 + hd_ - 1, gh = h0 + hh_ - 1, gw = w0 + hw_ - 1;
      if (live && hv < G6::Halo && (unsigned)gd < (unsigned)p.D && (unsigned)gh < (unsigned)p.H &&
          (unsigned)gw < (unsigned)p.W)
        voff = ((uint32_t)(((n * p.D + gd) * p.H + gh) * p.W + gw) * stride + cofs + (uint32_t)(pc & 1) * 8u) * 2u;
    }
    const bool dummy = j == G6::Pieces - 1 && j * G6::T + wave * 64 >= 2 * G6::Halo;
    const uint32_t lb = __builtin_amdgcn_readfirstlane(
        dummy ? lds0 + 2 * G6::Buf : lds0 + buf * G6::Buf + (wave * 64 + j * G6::T) * 16);
    dma16(first ? xr0 : xr1, lb, dummy ? kOOB : voff, 0);
    return !dummy && voff != kOOB ? 1u << j : 0u;
  };
  float* bnt = reinterpret_cast<float*>(lds + G6::BnOff);
  auto bn_apply = [&](int buf, int chunk, uint32_t pm) {
#pragma unroll
    for (int j = 0; j < G6::Pieces; ++j) {
      if (!((pm >> j) & 1)) continue;
      const int pc = tid + j * G6::T;
      u32x4_t* q = reinterpret_cast<u32x4_t*>(lds + buf * G6::Buf + pc * 16);
      const int c = chunk * 16 + (tid & 1) * 8;  // piece pc = tid + T j: its half is tid & 1
      const f32x4_t s0 = *reinterpret_cast<const f32x4_t*>(bnt + c), s1 = *reinterpret_cast<const f32x4_t*>(bnt + c + 4);
      const f32x4_t h0 = *reinterpret_cast<const f32x4_t*>(bnt + kBgBnMax + c);
      const f32x4_t h1 = *reinterpret_cast<const f32x4_t*>(bnt + kBgBnMax + c + 4);
      const float sc[8] = {s0[0], s0[1], s0[2], s0[3], s1[0], s1[1], s1[2], s1[3]};
      const float sh[8] = {h0[0], h0[1], h0[2], h0[3], h1[0], h1[1], h1[2], h1[3]};
      u32x4_t v = *q;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        v[i] = pack_bf16x2(bn_relu1(__uint_as_float(v[i] << 16), sc[2 * i], sh[2 * i]),
                           bn_relu1(__uint_as_float(v[i] & 0xffff0000u), sc[2 * i + 1], sh[2 * i + 1]));
      *q = v;
    }
  };
  if constexpr (BNIN) {
    if (tid < p.Cin) { bnt[tid] = p.isc[tid]; bnt[kBgBnMax + tid] = p.ish[tid]; }
    __syncthreads();
  }

  // B: pack16, (16-chunk c, step s) rows of Cout / 16 fragments of 1 KiB; this wave's NT
  // N-tiles are the workgroup's CO channels: bases off (+ 4 KiB) + immediates 0-3 KiB
  const int nchunk = p.Cin >> 4;  // (the pack's chunk count; SPLIT: this split's [cbeg, cend))
  const int cbeg = split * (SPLIT ? p.chunks_per_split : 0), cend = SPLIT ? cbeg + p.chunks_per_split : nchunk;
  const uint32_t step_bytes = (uint32_t)Cout * 64u;
  const i32x4_t wr = buffer_desc(p.w, (uint32_t)nchunk * kB6Steps * step_bytes);
  auto load_b = [&](s16x8_t (&dst)[NT], int chunk, int st, uint32_t boff) {
    const uint32_t off = boff + (uint32_t)(chunk * kB6Steps + st) * step_bytes;
#pragma unroll
    for (int h = 0; h < NT / 4; ++h) {
      bload16<0>(dst[4 * h + 0], wr, off + h * 4096u);
      bload16<1024>(dst[4 * h + 1], wr, off + h * 4096u);
      bload16<2048>(dst[4 * h + 2], wr, off + h * 4096u);
      bload16<3072>(dst[4 * h + 3], wr, off + h * 4096u);
    }
  };

  float* red = reinterpret_cast<float*>(lds + G6::RedOff);  // [wave][CO][mean, M2, n]
  float* bls = red + BD * CO * 3;
  if (tid < CO) bls[tid] = p.bias ? p.bias[co_base + tid] : 0.f;
  // outputs per 64-channel half h of the block: y0 below cy0, y1 from it (the dgrad's two Up3D
  // sources; cy0 % 64 == 0)
  auto ydst = [&](int h, long& ys, int& yc0) {
    const int cb = co_base + 64 * h;
    const bool to0 = cb < p.cy0;
    ys = to0 ? p.cy0 : Cout - p.cy0;
    yc0 = to0 ? cb : cb - p.cy0;
    return __builtin_amdgcn_make_buffer_rsrc(to0 ? p.y0 : p.y1, (short)0, (int)(p.nvox * ys * 2), 0x00020000);
  };
  char* slice = lds + G6::SliceOff + wave * (SPLIT ? 16 * G6::Row32 : G6::Slice);
  int nbdone = 0;

  f32x4_t acc[8][NT];
  constexpr int kB6Dist = b6_dist<BD, NT>();
  static_assert(kB6Steps % (kB6Dist + 1) == 0, "B ring index must continue across chunks");
  s16x8_t bset[kB6Dist + 1][NT];
  int box = slot;
  int n, d0, h0, w0;
  origin(box, n, d0, h0, w0);
  if (cend - cbeg <= 4)
    for (int i = 0; i < 2 * (slot & 3); ++i) __builtin_amdgcn_s_sleep(127);
  uint32_t pmask = 0;
#pragma unroll
  for (int j = 0; j < G6::Pieces; ++j) pmask |= stage_piece(n, d0, h0, w0, cbeg, 0, j, true, true);
  {
    const uint32_t boff0 = (uint32_t)(cob * NT * 1024 + lane * 16);
#pragma unroll
    for (int t = 0; t < kB6Dist; ++t) load_b(bset[t], cbeg, t, boff0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if constexpr (BNIN) bn_apply(0, 0, pmask);
  __syncthreads();
  int buf = 0;
  while (true) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
    const int nbx = box + nslot;
    const bool has_next = nbx < nbox;
    int nn = n, nd0 = d0, nh0 = h0, nw0 = w0;
    if (has_next) origin(nbx, nn, nd0, nh0, nw0);
    auto run_chunk = [&](int chunk, auto slack_tag) {
      constexpr bool Slack = decltype(slack_tag)::value;
      const bool last = chunk + 1 == cend;
      const bool live = !last || has_next;
      const int sn = last ? nn : n, sd = last ? nd0 : d0, sh = last ? nh0 : h0, sw = last ? nw0 : w0;
      const int schunk = last ? cbeg : chunk + 1;
      const int lo = opaque(lane);
      const uint32_t boff = (uint32_t)(cob * NT * 1024 + lo * 16);
      // A: this lane's halo row base -- box voxel (d = wave, h = 0, w = r16), its channel half
      // (g4 & 1) -- plus the row offset of its tap of the pair (g4 >> 1); M-tile mt = h-row mt
      // is an immediate (mt x 18 rows)
      const int r16 = lo & 15;  // the lane's voxel of an M-tile: h-row r16 / WB, w r16 % WB
      const uint32_t abase = lds0 + buf * G6::Buf +
                             (uint32_t)(((wave * GW::HH + r16 / WB) * GW::HW + r16 % WB) * 32 + ((lo >> 4) & 1) * 16);
      const bool hi_tap = (lo >> 5) & 1;
      // A fragment of (step st, M-tile mt); fragments are read two M-tiles ahead of their four
      // MFMAs through a 3-register rotation, across step boundaries (a deeper, per-step rolling
      // set made the compiler double-buffer it into spills)
      auto rd = [&](int st, int mt) {
        const uint32_t ad = abase + (uint32_t)(hi_tap ? b6_tapoff<WB>(2 * st + 1) : b6_tapoff<WB>(2 * st)) * 32u;
        return *reinterpret_cast<const LDS_AS s16x8_t*>((const LDS_AS char*)(uintptr_t)ad + mt * GW::MTR * 32);
      };
      s16x8_t ar[3];
      ar[0] = rd(0, 0);
      ar[1] = rd(0, 1);
      static_for<kB6Steps>([&](auto sc) {
        constexpr int st = decltype(sc)::value;
        constexpr int sn_ = st + kB6Dist;
        if constexpr (sn_ < kB6Steps) load_b(bset[sn_ % (kB6Dist + 1)], chunk, sn_, boff);
        else load_b(bset[sn_ % (kB6Dist + 1)], schunk, sn_ - kB6Steps, boff);
        if constexpr (st < G6::Pieces) {
          const uint32_t bits = stage_piece(sn, sd, sh, sw, schunk, buf ^ 1, st, live, last);
          if constexpr (BNIN) pmask = (st == 0 ? 0u : pmask) | bits;
        }
        s16x8_t (&b)[NT] = bset[st % (kB6Dist + 1)];
        constexpr int extra = (Slack && st < kB6Dist) ? (SPLIT ? G6::EpiStores32 : G6::EpiStores) : 0;
        vm_wait4<b6_wait<G6::Pieces, kB6Dist, NT>(st) + extra>(b);
        static_for<8>([&](auto mc) {
          constexpr int mt = decltype(mc)::value;
          constexpr int q = st * 8 + mt + 2;  // the fragment read now: position q (two ahead)
          if constexpr (q < kB6Steps * 8) ar[q % 3] = rd(q / 8, q % 8);
#pragma unroll
          for (int j = 0; j < NT; ++j) {
            if constexpr (kT) acc[mt][j] = mfma16(b[j], ar[(st * 8 + mt) % 3], acc[mt][j]);
            else acc[mt][j] = mfma16(ar[(st * 8 + mt) % 3], b[j], acc[mt][j]);
          }
        });
        // keep the order (1 read, NT MFMAs per M-tile) and every step's work in its step
#pragma unroll
        for (int mt = 0; mt < 8; ++mt) {
          if (st * 8 + mt + 2 < kB6Steps * 8) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // 1 DS read
          __builtin_amdgcn_sched_group_barrier(0x008, NT, 0);  // NT MFMA
        }
        __builtin_amdgcn_sched_barrier(0);
      });
      if (!last) vm_wait<NT * (kB6Steps - G6::Pieces)>();
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if constexpr (BNIN && (BG_ABL & 128) == 0) bn_apply(buf ^ 1, schunk, pmask);  // (128: ablation)
      __syncthreads();
      buf ^= 1;
    };
    run_chunk(cbeg, std::true_type{});
    for (int chunk = cbeg + 1; chunk < cend; ++chunk) run_chunk(chunk, std::false_type{});

    if constexpr (SPLIT) {
      // fp32 partial rows of this split: one M-tile at a time through the wave's slice (16 rows
      // of CO fp32), read back as whole 256-B voxel rows, 16-B stores
      const int lane_o = opaque(lane);
      const int rr = lane_o & 15, gg = lane_o >> 4;
      const long vbase = (((long)n * p.D + d0 + wave) * p.H + h0) * p.W + w0;
      const __amdgpu_buffer_rsrc_t ar = __builtin_amdgcn_make_buffer_rsrc(
          p.yacc, (short)0, (int)((long)nsplit * p.nvox * Cout * 4), 0x00020000);
#pragma unroll
      for (int mt = 0; mt < 8; ++mt) {
#pragma unroll
        for (int j = 0; j < NT; ++j) {
          if constexpr (kT) {  // lane (gg, rr): voxel rr, channels 16 j + 4 gg .. + 3
            *reinterpret_cast<f32x4_t*>(slice + rr * G6::Row32 + (16 * j + 4 * gg) * 4) = acc[mt][j];
          } else {
#pragma unroll
            for (int i = 0; i < 4; ++i)
              *reinterpret_cast<float*>(slice + (4 * gg + i) * G6::Row32 + (16 * j + rr) * 4) = acc[mt][j][i];
          }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int k = 0; k < CO / 16; ++k) {
          const int q = lane_o + 64 * k, vw = q >> 4, c4 = q & 15;
          const u32x4_t v = *reinterpret_cast<const u32x4_t*>(slice + vw * G6::Row32 + c4 * 16);
          const long vox = vbase + (long)(mt * (16 / WB) + vw / WB) * p.W + vw % WB;
          __builtin_amdgcn_raw_buffer_store_b128(v, ar, (int)((((long)split * p.nvox + vox) * Cout + co_base + c4 * 4) * 4),
                                                 0, 0);
        }
      }
      if (!has_next) break;
      box = nbx;
      n = nn; d0 = nd0; h0 = nh0; w0 = nw0;
      continue;
    }

    // ---- epilogue of this box: lane (g4, r16) holds, per (M-tile mt, N-tile j), voxels w =
    // 4 g4 + i (i < 4) of h-row mt, channel 16 j + r16.  One M-tile at a time through the wave's
    // own slice (16 rows of Row B): + bias, bf16; read back as whole 128-B half rows (NT / 2 x
    // 16 B per lane, each store instruction inside one 64-channel half), 16-B stores.
    // BatchNorm moments shifted by K (the running mean; the bias before the first box), per
    // channel over the wave's 128 voxels, Chan-merged per (wave, channel).
    if constexpr ((BG_ABL & 64) != 0) {  // ablation: no epilogue at all
#pragma unroll
      for (int mt = 0; mt < 8; ++mt)
#pragma unroll
        for (int j = 0; j < NT; ++j) asm volatile("" ::"v"(acc[mt][j]));
      if (!has_next) break;
      box = nbx;
      n = nn; d0 = nd0; h0 = nh0; w0 = nw0;
      continue;
    }
    if constexpr (kT) {
      // lane (gg, rr) holds, per (M-tile mt, N-tile j), voxel rr of h-row(s) mt and channels
      // 16 j + 4 gg + i (i < 4): + bias, bf16, one 8-B store.  BatchNorm moments shifted by K
      // (the running mean; the bias before the first box) summed over the lane's 8 M-tiles,
      // then over the 16 lanes of its DPP row (the wave's 128 voxels), Chan-merged per (wave,
      // channel) as below
      const int lane_o = opaque(lane);
      const int rr = lane_o & 15, gg = lane_o >> 4;
      const long vbase = (((long)n * p.D + d0 + wave) * p.H + h0) * p.W + w0;
      const bool relu = p.accumulate & PCMS_CONV_RELU;
      const bool want_stats = p.stats != nullptr;  // (the dgrads: none)
      long ys;
      int yc0;
      const auto yr = ydst(0, ys, yc0);
      const float rn = (float)nbdone * 128.f;
      constexpr float nb = 128.f;  // voxels per wave and box
      const float nnew = rn + nb;
      // statistics N-tile by N-tile (4 channels x 2 sums live), then the values M-tile by
      // M-tile through the wave's slice: one 8-B LDS write per (M-tile, N-tile), read back as
      // whole 128-B half rows for 16-B stores (register-direct 8-B stores touch 16 lines per
      // instruction and ran slower)
      float bias4[NT][4];
#pragma unroll
      for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i) bias4[j][i] = bls[16 * j + 4 * gg + i];
      if (want_stats) {
        // per-lane shifted sums of its 16 channels (m = 4 j + i) over its 8 voxels, then a
        // reduce-scatter over the 16 lanes of the row (4 DPP stages, halving the values each
        // time): lane rr ends with channel m = rr summed over the row's 128 voxels, and merges
        // that one channel
        // (channel pairs in packed fp32: v_pk_add_f32 / v_pk_fma_f32, the same IEEE results)
        float S1[4 * NT], S2[4 * NT];
#pragma unroll
        for (int j = 0; j < NT; ++j) {
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            const int c0 = 16 * j + 4 * gg + 2 * q;
            const float k0 = nbdone ? red[(wave * CO + c0) * 3] : bias4[j][2 * q];
            const float k1 = nbdone ? red[(wave * CO + c0 + 1) * 3] : bias4[j][2 * q + 1];
            const f32x2_t sh = {bias4[j][2 * q] - k0, bias4[j][2 * q + 1] - k1};
            f32x2_t s1 = {0.f, 0.f}, s2 = {0.f, 0.f};
#pragma unroll
            for (int mt = 0; mt < 8; ++mt) {
              const f32x2_t e = (f32x2_t){acc[mt][j][2 * q], acc[mt][j][2 * q + 1]} + sh;
              s1 += e;
              s2 = __builtin_elementwise_fma(e, e, s2);
            }
            S1[4 * j + 2 * q] = s1[0];
            S1[4 * j + 2 * q + 1] = s1[1];
            S2[4 * j + 2 * q] = s2[0];
            S2[4 * j + 2 * q + 1] = s2[1];
          }
        }
        auto stage = [&](auto nc, auto ctl, bool hi) __attribute__((always_inline)) {
          constexpr int h = decltype(nc)::value / 2;
          constexpr int c = decltype(ctl)::value;
#pragma unroll
          for (int k = 0; k < h; ++k) {
            const float k1 = hi ? S1[h + k] : S1[k], t1 = hi ? S1[k] : S1[h + k];
            const float k2 = hi ? S2[h + k] : S2[k], t2 = hi ? S2[k] : S2[h + k];
            S1[k] = k1 + __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, t1), c, 0xf, 0xf, true));
            S2[k] = k2 + __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, t2), c, 0xf, 0xf, true));
          }
        };
        static_assert(NT == 4, "16 channels per lane");
        stage(std::integral_constant<int, 16>{}, std::integral_constant<int, 0x140>{}, (rr & 8) != 0);  // 15 - r
        stage(std::integral_constant<int, 8>{}, std::integral_constant<int, 0x141>{}, (rr & 4) != 0);   // 7 - r
        stage(std::integral_constant<int, 4>{}, std::integral_constant<int, 0x4e>{}, (rr & 2) != 0);    // r ^ 2
        stage(std::integral_constant<int, 2>{}, std::integral_constant<int, 0xb1>{}, (rr & 1) != 0);    // r ^ 1
        const int ch = 16 * (rr >> 2) + 4 * gg + (rr & 3);
        float* rme = red + (wave * CO + ch) * 3;
        const float K = nbdone ? rme[0] : bls[ch];
        const float s1 = S1[0], s2 = S2[0];
        const float mbox = K + s1 / nb;
        const float m2b = fmaxf(s2 - s1 * s1 / nb, 0.f);
        const float rmean = nbdone ? rme[0] : 0.f, rm2 = nbdone ? rme[1] : 0.f;
        const float delta = mbox - rmean;
        rme[0] = rmean + delta * (nb / nnew);
        rme[1] = rm2 + m2b + delta * delta * (rn * nb / nnew);
        rme[2] = nnew;
      }
#pragma unroll
      for (int mt = 0; mt < 8; ++mt) {
#pragma unroll
        for (int j = 0; j < NT; ++j) {
          uint32_t o[2];
#pragma unroll
          for (int k = 0; k < 2; ++k) {
            f32x2_t a = (f32x2_t){acc[mt][j][2 * k], acc[mt][j][2 * k + 1]} +
                        (f32x2_t){bias4[j][2 * k], bias4[j][2 * k + 1]};
            if (relu) a = (f32x2_t){fmaxf(a[0], 0.f), fmaxf(a[1], 0.f)};
            o[k] = __builtin_bit_cast(uint32_t, __builtin_convertvector(a, bf16x2_t));
          }
          *reinterpret_cast<u32x2_t*>(slice + rr * G6::Row + (16 * j + 4 * gg) * 2) = (u32x2_t){o[0], o[1]};
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int k = 0; k < NT / 2; ++k) {
          const int vw = (k * 64 + lane_o) >> 3, c8 = lane_o & 7;
          const u32x4_t v = *reinterpret_cast<const u32x4_t*>(slice + vw * G6::Row + c8 * 16);
          const long vox = vbase + (long)(mt * (16 / WB) + vw / WB) * p.W + vw % WB;
          if constexpr ((BG_ABL & 2) == 0)
            __builtin_amdgcn_raw_buffer_store_b128(v, yr, (int)((vox * ys + yc0 + c8 * 8) * 2), 0, 0);
          else
            asm volatile("" ::"v"(v), "v"((int)vox));
        }
      }
      ++nbdone;
      if (!has_next) break;
      box = nbx;
      n = nn; d0 = nd0; h0 = nh0; w0 = nw0;
      continue;
    }
    const int lane_o = opaque(lane);
    const int rr = lane_o & 15, gg = lane_o >> 4;
    const long plane = (long)p.H * p.W;
    const long vbase = (((long)n * p.D + d0 + wave) * p.H + h0) * p.W + w0;
    const bool relu = p.accumulate & PCMS_CONV_RELU;
    float bias_j[NT], K0[NT], S1[NT], S2[NT];
    const float rn = (float)nbdone * 128.f;
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      bias_j[j] = bls[16 * j + rr];
      K0[j] = nbdone ? red[(wave * CO + 16 * j + rr) * 3] : bias_j[j];
      S1[j] = 0.f;
      S2[j] = 0.f;
    }
#pragma unroll
    for (int mt = 0; mt < 8; ++mt) {
#pragma unroll
      for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float v0 = acc[mt][j][i];
          if constexpr ((BG_ABL & 32) == 0)
            *reinterpret_cast<bf16_t*>(slice + (4 * gg + i) * G6::Row + (16 * j + rr) * 2) =
                f2bf(relu ? fmaxf(v0 + bias_j[j], 0.f) : v0 + bias_j[j]);
          else
            asm volatile("" ::"v"(v0));
          const float e0 = v0 + (bias_j[j] - K0[j]);
          S1[j] += e0;
          S2[j] = fmaf(e0, e0, S2[j]);
        }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int k = 0; k < NT / 2; ++k) {
        const int h = k >> 1, vw = ((k & 1) * 64 + lane_o) >> 3, c8 = lane_o & 7;
        long ys;
        int yc0;
        const auto yr = ydst(h, ys, yc0);
        const u32x4_t v = *reinterpret_cast<const u32x4_t*>(slice + vw * G6::Row + (h * 8 + c8) * 16);
        const long vox = vbase + (long)(mt * (16 / WB) + vw / WB) * p.W + vw % WB;
        if constexpr ((BG_ABL & 2) == 0)
          __builtin_amdgcn_raw_buffer_store_b128(v, yr, (int)((vox * ys + yc0 + c8 * 8) * 2), 0, 0);
        else
          asm volatile("" ::"v"(v), "v"((int)vox));
      }
      (void)plane;
    }
    {
      constexpr float nb = 128.f;  // voxels per wave and box
      const float nnew = rn + nb;
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        float s1 = S1[j], s2 = S2[j];
        s1 += __shfl_xor(s1, 16, 64);
        s2 += __shfl_xor(s2, 16, 64);
        s1 += __shfl_xor(s1, 32, 64);
        s2 += __shfl_xor(s2, 32, 64);
        const float mbox = K0[j] + s1 / nb;
        const float m2b = fmaxf(s2 - s1 * s1 / nb, 0.f);
        float* rme = red + (wave * CO + 16 * j + rr) * 3;
        const float rmean = nbdone ? rme[0] : 0.f, rm2 = nbdone ? rme[1] : 0.f;
        const float delta = mbox - rmean;
        if (gg == 0) {
          rme[0] = rmean + delta * (nb / nnew);
          rme[1] = rm2 + m2b + delta * delta * (rn * nb / nnew);
          rme[2] = nnew;
        }
      }
      ++nbdone;
    }
    if (!has_next) break;
    box = nbx;
    n = nn; d0 = nd0; h0 = nh0; w0 = nw0;
  }

  if (SPLIT || !p.stats) return;
  __syncthreads();
  if (tid < CO) {
    float S = 0.f, Nn = 0.f;
#pragma unroll
    for (int w = 0; w < BD; ++w) {
      S += red[(w * CO + tid) * 3] * red[(w * CO + tid) * 3 + 2];
      Nn += red[(w * CO + tid) * 3 + 2];
    }
    const float m = S / Nn;
    float M2 = 0.f;
#pragma unroll
    for (int w = 0; w < BD; ++w) {
      const float c = red[(w * CO + tid) * 3 + 2];
      const float d = red[(w * CO + tid) * 3] - m;
      M2 += red[(w * CO + tid) * 3 + 1] + c * d * d;
    }
    float* st = p.stats + ((long)slot * Cout + co_base + tid) * 2;
    st[0] = S;
    st[1] = M2;
    if (tid == 0 && cob == 0) p.stats[(long)nslot * Cout * 2 + slot] = Nn;
  }
}

// pack16 layout (conv3_fwd_b16_kernel's B operand): element (16-chunk c, tap pair s, row j,
// lane group g, element e) = w[j][16 c + 8 (g & 1) + e][tap 2 s + (g >> 1)] (tap 27: zero), in
// 1 KiB blocks (c, s, j / 16) of lanes l = 16 g + j % 16 -- the v_mfma_f32_16x16x32_bf16 B
// fragment of that (tap pair, 16-row tile).  J % 16 == 0, Kdim % 16 == 0.
__host__ __device__ inline long pack16_off(int c, int s, int j, int g, int J) {
  return (((long)c * kB6Steps + s) * (J >> 4) + (j >> 4)) * 512 + (g * 16 + (j & 15)) * 8;
}
// Both pack16 forms of the convs of a table, from the fp32 master (one block per 32 co x 32 ci
// tile, as pack_conv3_bf16_both_kernel): rows int64[8] = {weight ptr, Cout, Cin, fwd16 ptr (or
// 0), dgrad16 ptr (or 0), first tile, 0, 0}.  fwd16: J = Cout rows, k = Cin; dgrad16: J = Cin
// rows, k = Cout, taps mirrored (the dgrad conv is the transposed, flipped forward).
__global__ void __launch_bounds__(256) pack16_conv3_kernel(const long long* tab, int ntab) {
  __shared__ __attribute__((aligned(16))) uint16_t tb[32 * 864];
  int ei = 0;
  while (ei + 1 < ntab && tab[8 * (ei + 1) + 5] <= (long long)blockIdx.x) ++ei;
  const long long* e = tab + 8 * ei;
  const float* w = reinterpret_cast<const float*>(e[0]);
  const int Cout = (int)e[1], Cin = (int)e[2];
  bf16_t* fwd = reinterpret_cast<bf16_t*>(e[3]);
  bf16_t* dgr = reinterpret_cast<bf16_t*>(e[4]);
  const int local = blockIdx.x - (int)e[5];
  const int j0 = (local % (Cout / 32)) * 32, ci0 = (local / (Cout / 32)) * 32;
  // all 27 loads of a thread in flight at once (as pack_conv3_bf16_both_kernel)
  f32x4_t v[27];
#pragma unroll
  for (int i = 0; i < 27; ++i) {
    const int q4 = threadIdx.x + i * 256, run = q4 / 216, q = q4 % 216;
    v[i] = __builtin_nontemporal_load(reinterpret_cast<const f32x4_t*>(w + ((long)(j0 + run) * Cin + ci0) * 27) + q);
  }
#pragma unroll
  for (int i = 0; i < 27; ++i) {
    const int q4 = threadIdx.x + i * 256, run = q4 / 216, q = q4 % 216;
    uint2 o;
    o.x = pack_bf16x2(v[i][0], v[i][1]);
    o.y = pack_bf16x2(v[i][2], v[i][3]);
    *reinterpret_cast<uint2*>(tb + run * 864 + 4 * q) = o;
  }
  __syncthreads();
  pack16_tile_store(tb, fwd, dgr, j0, ci0, Cout, Cin);
}

__device__ void pack16_tile_store(const uint16_t* tb, bf16_t* fwd, bf16_t* dgr, int j0, int ci0, int Cout, int Cin) {
  // 2 chunks x 14 steps x 2 row tiles x 64 lanes = 3584 16-B pieces per direction
  for (int it = threadIdx.x; it < 2 * 3584; it += 256) {
    const int dir = it / 3584, q = it % 3584;
    bf16_t* out = dir ? dgr : fwd;
    if (!out) continue;
    const int l = q & 63, rt = (q >> 6) & 1, st = (q >> 7) % kB6Steps, cc = (q >> 7) / kB6Steps;
    const int g = l >> 4, jl = rt * 16 + (l & 15);             // row within the 32-row tile
    const int tap = 2 * st + (g >> 1);
    uint32_t o[4];
#pragma unroll
    for (int ee = 0; ee < 4; ++ee) {
      uint32_t v2 = 0;
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const int kl = cc * 16 + 8 * (g & 1) + 2 * ee + hh;  // k within the 32-wide tile
        uint16_t v = 0;
        if (tap < 27) v = dir ? tb[kl * 864 + jl * 27 + (26 - tap)] : tb[jl * 864 + kl * 27 + tap];
        v2 |= (uint32_t)v << (16 * hh);
      }
      o[ee] = v2;
    }
    const int J = dir ? Cin : Cout;
    const int jg = (dir ? ci0 : j0) + jl;                      // global row
    const int cg = ((dir ? j0 : ci0) >> 4) + cc;               // global 16-chunk
    *reinterpret_cast<u32x4_t*>(out + pack16_off(cg, st, jg, g, J)) = (u32x4_t){o[0], o[1], o[2], o[3]};
  }
}

}  // namespace

// big-box forward: bf16, whole 8x8x16 boxes, 16-channel chunks of both sources, enough boxes
// to give every CU one (pcms_conv3_big_min_boxes), every byte offset inside a 32-bit voffset
static int g_big_min_boxes = 256;
static int g_conv_mtw2 = 1;  // boxes of <= 256 voxels on 2 M-tiles per wave (A/B switch)
static int g_fwd_box_vol = 512;  // general forward / dgrad box volume (512 or 256; A/B switch)
static int g_big_max_wgs = 0;  // persistent grid cap (0: one workgroup per CU)
static bool big_fwd_ok(int dtype, int N, int D, int H, int W, int c0, int c1) {
  if (dtype != PCMS_BF16 || D % kBgBD || H % 8 || W % 16 || c0 % 16 || c1 % 16 || c0 < 16) return false;
  const long nvox = (long)N * D * H * W;
  if ((long)N * (D / kBgBD) * (H / 8) * (W / 16) < g_big_min_boxes) return false;
  return nvox < (1L << 30) && nvox * std::max(c0, c1) * 2 < (long)kOOB;
}
// (the output descriptor additionally needs nvox * Cout * 2 < 2^31: checked at launch)
// box slots of the persistent grid (= BatchNorm stats rows): each slot's workgroups (one
// per 64-channel block) walk boxes slot, slot + nslot, ...
static int big_slots(int N, int D, int H, int W, int Cout) {
  const int nbox = N * (D / kBgBD) * (H / 8) * (W / 16);
  const int G = g_big_max_wgs > 0 ? g_big_max_wgs : device_cus();
  return std::max(1, std::min(nbox, G / (Cout / 64)));
}

extern "C" {

// Returns the m-block count (workgroups along M) of the general fwd kernel for a grid
// (an upper bound on every fwd path's BatchNorm row count; sizes the split decision).
int pcms_conv3_mblocks(int N, int D, int H, int W) {
  Box b = fwd_box(D, H, W, g_fwd_box_vol);
  return N * cdiv(D, 1 << b.lbd) * cdiv(H, 1 << b.lbh) * cdiv(W, 1 << b.lbw);
}

// BatchNorm partial rows an unsplit pcms_conv3_fwd with these sources writes
int pcms_conv3_fwd_rows(int dtype, int N, int D, int H, int W, int c0, int c1, int Cout) {
  if (Cout % 64 == 0 && big_fwd_ok(dtype, N, D, H, W, c0, c1) && (long)N * D * H * W * Cout * 2 < (long)kOOB)
    return big_slots(N, D, H, W, Cout);
  return pcms_conv3_mblocks(N, D, H, W);
}

// Minimum box count for the big-box forward (tests lower it to reach small grids);
// v <= 0 only queries.  Returns the previous value.
int pcms_conv3_big_min_boxes(int v) {
  const int old = g_big_min_boxes;
  if (v > 0) g_big_min_boxes = v;
  return old;
}

// Workgroup cap of the persistent big-box grid (tests lower it so each workgroup walks
// several boxes); 0 restores one per CU, v < 0 only queries.  Returns the previous value.
int pcms_conv3_big_max_wgs(int v) {
  const int old = g_big_max_wgs;
  if (v >= 0) g_big_max_wgs = v;
  return old;
}

// general-kernel boxes of <= 256 voxels on four waves of 2 M-tiles (1) or two of 4 (0);
// v < 0 queries; returns the previous setting
// general-kernel forward / dgrad box volume: 512 or 256 voxels; v <= 0 queries; returns the
// previous setting (A/B switch: set before any workspace query)
int pcms_conv3_fwd_box_vol(int v) {
  const int old = g_fwd_box_vol;
  if (v == 256 || v == 512) g_fwd_box_vol = v;
  return old;
}

int pcms_conv3_small_box_mtw2(int v) {
  const int old = g_conv_mtw2;
  if (v >= 0) g_conv_mtw2 = v;
  return old;
}

int pcms_conv3_chunk(int dtype) {
  return dtype == PCMS_BF16 ? Traits<bf16_t>::CK : dtype == PCMS_F32X3 ? Traits<x3_t>::CK : Traits<x6_t>::CK;
}

// elements (of the activation dtype: bf16, or fp32 for both split modes) of one conv weight
// pack with J output rows and Kdim input channels: [ceil(Kdim / CK)][27][J][WK] bf16
int pcms_conv3_pack_elems(int dtype, int J, int Kdim) {
  const int ck = pcms_conv3_chunk(dtype);
  const int wk = dtype == PCMS_BF16 ? Traits<bf16_t>::WK : dtype == PCMS_F32X3 ? Traits<x3_t>::WK : Traits<x6_t>::WK;
  const long bf16s = (long)cdiv(Kdim, ck) * 27 * J * wk;
  return (int)(dtype == PCMS_BF16 ? bf16s : bf16s / 2);
}

// forward and dgrad packs together (one weight read); other shapes / dtypes: the two packs
int pcms_conv3_pack2(int dtype, const float* w, void* fwd, void* dgrad, int Cout, int Cin, hipStream_t s) {
  if (dtype == PCMS_BF16 && Cin % 32 == 0 && Cout % 32 == 0) {
    hipLaunchKernelGGL(pack_conv3_bf16_both_kernel, dim3(Cout / 32, Cin / 32), dim3(256), 0, s, w, (bf16_t*)fwd,
                       (bf16_t*)dgrad, Cout, Cin);
    PCMS_CHECK_LAUNCH();
  }
  const int rc = pcms_conv3_pack(dtype, w, fwd, Cout, Cin, 0, s);
  return rc ? rc : pcms_conv3_pack(dtype, w, dgrad, Cout, Cin, 1, s);
}

// Adam over the conv weights of a table (see adam_pack_conv3_kernel; every entry has
// Cout % 32 == Cin % 32 == 0 and 16-B aligned offsets), writing both bf16 packs.
int pcms_adam_pack_conv3(float* p, float* g, float* m, float* v, const long long* table, int ntab, int ntiles,
                         float step_size, float b1, float b2, float eps, float wd, float bc2_sqrt, float gscale,
                         const float* gmul, hipStream_t s) {
  if (ntab <= 0 || ntiles <= 0) return 0;
  const AdamCoef c{step_size, b1, b2, eps, wd, bc2_sqrt, gscale};
  hipLaunchKernelGGL(adam_pack_conv3_kernel, dim3(ntiles), dim3(256), 0, s, p, g, m, v, table, ntab, c, gmul);
  PCMS_CHECK_LAUNCH();
}

// the same for the fp32 build: both bf16x6 packs (pcms_conv3_pack dtype 0 layouts); one tile
// per 32 co x 16 ci (ntiles = sum of Cout / 32 x Cin / 16)
int pcms_adam_pack_conv3_x6(float* p, float* g, float* m, float* v, const long long* table, int ntab, int ntiles,
                            float step_size, float b1, float b2, float eps, float wd, float bc2_sqrt, float gscale,
                            const float* gmul, hipStream_t s) {
  if (ntab <= 0 || ntiles <= 0) return 0;
  const AdamCoef c{step_size, b1, b2, eps, wd, bc2_sqrt, gscale};
  hipLaunchKernelGGL(adam_pack_conv3_x6_kernel, dim3(ntiles), dim3(256), 0, s, p, g, m, v, table, ntab, c, gmul);
  PCMS_CHECK_LAUNCH();
}

int pcms_conv3_pack(int dtype, const float* w, void* out, int Cout, int Cin, int flip, hipStream_t s) {
  const int CK = pcms_conv3_chunk(dtype);
  const int J = flip ? Cin : Cout;
  const int Kdim = flip ? Cout : Cin;
  if (dtype == PCMS_BF16 && J % 32) return -1;  // fragment-major rows come in 32-row tiles
  dim3 grid(cdiv(J, 8), cdiv(Kdim, CK));
  if (dtype == PCMS_BF16 && Kdim % 32 == 0 && J % 8 == 0)
    hipLaunchKernelGGL(pack_conv3_bf16_kernel, grid, dim3(256), 0, s, w, (bf16_t*)out, Cout, Cin, flip);
  else if (dtype == PCMS_BF16)
    hipLaunchKernelGGL((pack_conv3_kernel<bf16_t, 32>), grid, dim3(256), 0, s, w, (bf16_t*)out, Cout, Cin, flip);
  else if (dtype == PCMS_F32X3)
    hipLaunchKernelGGL((pack_conv3_kernel<x3_t, 16>), grid, dim3(256), 0, s, w, (x3_t*)out, Cout, Cin, flip);
  else
    hipLaunchKernelGGL((pack_conv3_kernel<x6_t, 8>), grid, dim3(256), 0, s, w, (x6_t*)out, Cout, Cin, flip);
  PCMS_CHECK_LAUNCH();
}

// Input-channel splits a split-K launch with `splits` requested actually uses (whole
// chunks per split): the slab count of yacc and of pcms_split_epilogue.
int pcms_conv3_splits(int dtype, int Cin, int splits) {
  const int nchunk = cdiv(Cin, pcms_conv3_chunk(dtype));
  splits = std::max(1, std::min(splits, nchunk));
  return cdiv(nchunk, cdiv(nchunk, splits));
}

// Forward (or dgrad) 3x3x3 conv. See Conv3Params.  splits > 1: every split writes its fp32
// partial sums into its own slab of yacc [splits][N*D*H*W][Cout] (plain stores, no zeroing
// needed); pcms_split_epilogue then sums the slabs in split order (deterministic), adds the
// bias, converts, and forms the BN statistics.
static int conv3_fwd_any(int dtype, const void* x0, int c0, const void* x1, int c1, const float* isc,
                         const float* ish, const void* wpack, const float* bias, void* y0, void* y1, int cy0,
                         float* yacc, float* stats, int flags, int N, int D, int H, int W, int Cout, int splits,
                         hipStream_t s);

int pcms_conv3_fwd(int dtype, const void* x0, int c0, const void* x1, int c1,
                   const void* wpack, const float* bias, void* y0, void* y1, int cy0,
                   float* yacc, float* stats, int flags,
                   int N, int D, int H, int W, int Cout, int splits, hipStream_t s) {
  return conv3_fwd_any(dtype, x0, c0, x1, c1, nullptr, nullptr, wpack, bias, y0, y1, cy0, yacc, stats, flags, N, D,
                       H, W, Cout, splits, s);
}

// the same with the input's BatchNorm + ReLU applied in the staging path: the conv of
// relu(x * isc + ish) (bf16, one source of <= 128 channels, the big-box shapes; -5 otherwise)
int pcms_conv3_fwd_bnin(int dtype, const void* x, int cin, const float* isc, const float* ish, const void* wpack,
                        const float* bias, void* y, float* stats, int N, int D, int H, int W, int Cout,
                        hipStream_t s) {
  if (!isc || !ish || cin > kBgBnMax || dtype != PCMS_BF16) return -1;
  return conv3_fwd_any(dtype, x, cin, nullptr, 0, isc, ish, wpack, bias, y, nullptr, Cout, nullptr, stats, 0, N, D,
                       H, W, Cout, 1, s);
}

// ---- 16x16x32 big-box path (conv3_fwd_b16_kernel) ----
// box depth pcms_conv3_fwd16 runs a conv with: 8 where its 8-deep boxes (x 64-channel blocks)
// fill every CU (levels 0-1; level 2's 512-channel outputs), else 4 where 4-deep boxes do
// (level 2's 256-channel outputs: one wave per SIMD, profiles/r5_deep_ab.txt), else 0
static bool b16_shape_ok(int bd, int N, int D, int H, int W, int c0, int c1) {
  const long nvox = (long)N * D * H * W;
  return D % bd == 0 && H % 8 == 0 && W % 16 == 0 && c0 % 16 == 0 && c1 % 16 == 0 && c0 >= 16 &&
         nvox < (1L << 30) && nvox * std::max(c0, c1) * 2 < (long)kOOB;
}
struct B16Cfg { int bd, nt; };
// 128-channel blocks on 4-deep boxes (B6G<4, 8>) where Cout allows and they fill the CUs (A/B
// switch pcms_conv3_b16_nt8; off: 12-20 % slower than 64-channel blocks on 8-deep boxes at
// every level-0/1 shape despite a 5-12 % higher clock -- one wave per SIMD with 64 MFMAs per
// k-step cannot hide its B fetches, profiles/r5_nt8_ab.txt)
static int g_b16_nt8 = 0;
static B16Cfg b16_config(int N, int D, int H, int W, int c0, int c1, int Cout) {
  if (Cout % 64 || (long)N * D * H * W * Cout * 2 >= (long)kOOB) return {0, 0};
  const long nb8 = (long)N * (D / 8) * (H / 8) * (W / 16), nb4 = (long)N * (D / 4) * (H / 8) * (W / 16);
  const long ncob = Cout / 64;
  if (g_b16_nt8 && Cout % 128 == 0 && b16_shape_ok(4, N, D, H, W, c0, c1) && nb4 * (Cout / 128) >= g_big_min_boxes)
    return {4, 8};
  if (big_fwd_ok(PCMS_BF16, N, D, H, W, c0, c1)) return {8, 4};
  if (b16_shape_ok(8, N, D, H, W, c0, c1) && nb8 * ncob >= g_big_min_boxes) return {8, 4};
  if (b16_shape_ok(4, N, D, H, W, c0, c1) && nb4 * ncob >= g_big_min_boxes) return {4, 4};
  return {0, 0};
}
static int b16_slots(B16Cfg c, int N, int D, int H, int W, int Cout) {
  const int nbox = N * (D / c.bd) * (H / 8) * (W / 16);
  const int G = g_big_max_wgs > 0 ? g_big_max_wgs : device_cus();
  return std::max(1, std::min(nbox, G / (Cout / (16 * c.nt))));
}

// 1 when pcms_conv3_fwd16 runs this conv (bf16, one split); the engine keeps a pack16 for
// such convs
int pcms_conv3_big16_ok(int N, int D, int H, int W, int c0, int c1, int Cout) {
  return b16_config(N, D, H, W, c0, c1, Cout).bd ? 1 : 0;
}
// 128-channel blocks of the 16x16x32 kernel on (1) or off (0); v < 0 queries; returns the
// previous setting (set before any workspace query: it changes pcms_conv3_fwd16_rows)
int pcms_conv3_b16_nt8(int v) {
  const int old = g_b16_nt8;
  if (v >= 0) g_b16_nt8 = v;
  return old;
}
// BatchNorm partial rows pcms_conv3_fwd16 writes for this conv (0: not a fwd16 shape)
int pcms_conv3_fwd16_rows(int N, int D, int H, int W, int c0, int c1, int Cout) {
  const B16Cfg c = b16_config(N, D, H, W, c0, c1, Cout);
  return c.bd ? b16_slots(c, N, D, H, W, Cout) : 0;
}
int pcms_conv3_pack16_elems(int J, int Kdim) { return (J % 16 || Kdim % 16) ? -1 : (Kdim / 16) * kB6Steps * J * 32; }
// pack16 forms (fwd16: rows = Cout, k = Cin; dgrad16: rows = Cin, k = Cout, taps mirrored) of the
// convs of a table: int64 rows {weight ptr, Cout, Cin, fwd16 ptr or 0, dgrad16 ptr or 0, first
// tile, 0, 0}, one tile per 32 co x 32 ci (ntiles = sum of Cout / 32 x Cin / 32)
int pcms_conv3_pack16(const long long* table, int ntab, int ntiles, hipStream_t s) {
  if (ntab <= 0 || ntiles <= 0) return 0;
  hipLaunchKernelGGL(pack16_conv3_kernel, dim3(ntiles), dim3(256), 0, s, table, ntab);
  PCMS_CHECK_LAUNCH();
}
// y = conv(x) + bias on the 16x16x32 big-box kernel (wpack16 = a pcms_conv3_pack16 form);
// arguments as pcms_conv3_fwd with splits = 1; isc / ish != NULL: the input's BatchNorm + ReLU
// applied in the staging (as pcms_conv3_fwd_bnin; one source of <= 128 channels).  -5 when
// pcms_conv3_big16_ok is 0.
int pcms_conv3_fwd16(const void* x0, int c0, const void* x1, int c1, const float* isc, const float* ish,
                     const void* wpack16, const float* bias, void* y0, void* y1, int cy0, float* stats, int flags,
                     int N, int D, int H, int W, int Cout, hipStream_t s) {
  const B16Cfg cf = b16_config(N, D, H, W, c0, c1, Cout);
  const int bd = cf.bd;
  if (!bd || (c1 > 0 && x1 == nullptr)) return -5;
  if (isc && (c1 != 0 || c0 > kBgBnMax || !ish)) return -1;
  if (stats && flags) return -6;
  if (flags & ~PCMS_CONV_RELU) return -8;
  if (y1 == nullptr) cy0 = Cout;
  if (cy0 % 64 != 0 && cy0 != Cout) return -2;
  Conv3Params p;
  p.x0 = x0; p.x1 = x1; p.c0 = c0; p.c1 = c1;
  p.isc = isc; p.ish = ish;
  p.w = wpack16; p.bias = bias; p.y0 = y0; p.y1 = y1; p.cy0 = cy0;
  p.yacc = nullptr; p.stats = stats; p.accumulate = flags;
  p.N = N; p.D = D; p.H = H; p.W = W; p.Cin = c0 + c1; p.Cout = Cout;
  p.nvox = (long)N * D * H * W;
  p.nchunk = p.Cin / 16; p.chunks_per_split = p.nchunk;
  p.nbd = D / bd; p.nbh = H / 8; p.nbw = W / 16;
  const int nslot = b16_slots(cf, N, D, H, W, Cout);
  auto kern = cf.nt == 8 ? (isc ? conv3_fwd_b16_kernel<true, 4, 8> : conv3_fwd_b16_kernel<false, 4, 8>)
              : bd == 8  ? (isc ? conv3_fwd_b16_kernel<true, 8> : conv3_fwd_b16_kernel<false, 8>)
                         : (isc ? conv3_fwd_b16_kernel<true, 4> : conv3_fwd_b16_kernel<false, 4>);
  const int ldsb = cf.nt == 8 ? (isc ? B6G<4, 8>::LdsBn : B6G<4, 8>::Lds)
                   : bd == 8  ? (isc ? B6G<8>::LdsBn : B6G<8>::Lds)
                              : (isc ? B6G<4>::LdsBn : B6G<4>::Lds);
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, ldsb);
  hipLaunchKernelGGL(kern, dim3(nslot * (Cout / (16 * cf.nt))), dim3(bd * 64), ldsb, s, p,
                     (uint32_t)(p.nvox * c0 * 2), (uint32_t)(p.nvox * c1 * 2));
  PCMS_CHECK_LAUNCH();
}

// ---- split-K 16x16x32 form for level 3 (W = 8 rows): boxes of 4 d x 16 h x 8 w ----
// the split count pcms_conv3_fwd16_split uses for this conv (0: not such a shape -- whole
// 4-deep W8 boxes, fewer than 256 (box, 64-channel block) items, and a power-of-two split
// of the 16-channel chunks that brings them to >= 256 workgroups)
int pcms_conv3_fwd16_split_ok(int N, int D, int H, int W, int c0, int c1, int Cout) {
  const long nvox = (long)N * D * H * W;
  if (Cout % 64 || D % 4 || H % 16 || W % 8 || c0 % 16 || c1 % 16 || c0 < 16) return 0;
  if (nvox >= (1L << 30) || nvox * std::max(std::max(c0, c1), Cout) * 2 >= (long)kOOB) return 0;
  const long items = (long)N * (D / 4) * (H / 16) * (W / 8) * (Cout / 64);
  const int nchunk = (c0 + c1) / 16;
  if (items >= g_big_min_boxes) return 0;
  int sp = 1;
  while (items * sp < g_big_min_boxes && nchunk % (2 * sp) == 0) sp *= 2;
  if (sp == 1 || (long)sp * nvox * Cout * 4 >= (long)kOOB) return 0;
  return sp;
}

// yacc[split][vox][Cout] fp32 = this split's partial sums (no bias, no statistics; sum them
// with pcms_split_epilogue(yacc, splits, ...)); splits = pcms_conv3_fwd16_split_ok(...), -5 if
// that is 0
int pcms_conv3_fwd16_split(const void* x0, int c0, const void* x1, int c1, const void* wpack16, float* yacc,
                           int N, int D, int H, int W, int Cout, int splits, hipStream_t s) {
  if (splits < 2 || splits != pcms_conv3_fwd16_split_ok(N, D, H, W, c0, c1, Cout) || (c1 > 0 && x1 == nullptr))
    return -5;
  Conv3Params p;
  p.x0 = x0; p.x1 = x1; p.c0 = c0; p.c1 = c1;
  p.isc = nullptr; p.ish = nullptr;
  p.w = wpack16; p.bias = nullptr; p.y0 = nullptr; p.y1 = nullptr; p.cy0 = Cout;
  p.yacc = yacc; p.stats = nullptr; p.accumulate = 0;
  p.N = N; p.D = D; p.H = H; p.W = W; p.Cin = c0 + c1; p.Cout = Cout;
  p.nvox = (long)N * D * H * W;
  p.nchunk = p.Cin / 16; p.chunks_per_split = p.nchunk / splits;
  p.nbd = D / 4; p.nbh = H / 16; p.nbw = W / 8;
  const int nbox = N * p.nbd * p.nbh * p.nbw;
  const int G = g_big_max_wgs > 0 ? g_big_max_wgs : device_cus();
  const int nslot = std::max(1, std::min(nbox, G / ((Cout / 64) * splits)));
  auto kern = conv3_fwd_b16_kernel<false, 4, 4, 8, true>;
  const int ldsb = B6G<4>::LdsSplit;
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, ldsb);
  hipLaunchKernelGGL(kern, dim3(nslot * (Cout / 64) * splits), dim3(256), ldsb, s, p,
                     (uint32_t)(p.nvox * c0 * 2), (uint32_t)(p.nvox * c1 * 2));
  PCMS_CHECK_LAUNCH();
}

}  // extern "C"

static int conv3_fwd_any(int dtype, const void* x0, int c0, const void* x1, int c1, const float* isc,
                         const float* ish, const void* wpack, const float* bias, void* y0, void* y1, int cy0,
                         float* yacc, float* stats, int flags, int N, int D, int H, int W, int Cout, int splits,
                         hipStream_t s) {
  const int accumulate = flags & PCMS_CONV_ACCUMULATE;
  const int Cin = c0 + c1;
  const int CK = pcms_conv3_chunk(dtype);
  const int VEC = dtype == PCMS_BF16 ? 8 : 4;
  if (Cout % 64 != 0 || c0 % VEC != 0 || c1 % VEC != 0 || (c1 > 0 && x1 == nullptr)) return -1;
  if (stats && flags) return -6;  // BN statistics describe a fresh, pre-activation output only
  if (flags & ~(PCMS_CONV_ACCUMULATE | PCMS_CONV_RELU)) return -8;
  if (y1 == nullptr) cy0 = Cout;
  if (cy0 % 64 != 0 && cy0 != Cout) return -2;
  Box b = fwd_box(D, H, W, g_fwd_box_vol);
  Conv3Params p;
  p.x0 = x0; p.x1 = x1; p.c0 = c0; p.c1 = c1;
  p.isc = isc; p.ish = ish;
  p.w = wpack; p.bias = bias; p.y0 = y0; p.y1 = y1; p.cy0 = cy0;
  p.yacc = splits > 1 ? yacc : nullptr;
  p.stats = stats; p.accumulate = flags;
  p.N = N; p.D = D; p.H = H; p.W = W; p.Cin = Cin; p.Cout = Cout;
  p.nvox = (long)N * D * H * W;
  p.nchunk = cdiv(Cin, CK);
  if (splits < 1) splits = 1;
  if (splits > p.nchunk) splits = p.nchunk;
  p.chunks_per_split = cdiv(p.nchunk, splits);
  splits = cdiv(p.nchunk, p.chunks_per_split);
  if (splits > 1 && yacc == nullptr) return -3;
  p.lbd = b.lbd; p.lbh = b.lbh; p.lbw = b.lbw;
  p.nbd = cdiv(D, 1 << b.lbd); p.nbh = cdiv(H, 1 << b.lbh); p.nbw = cdiv(W, 1 << b.lbw);
  if (splits > 1) p.yacc = yacc;
  if (splits == 1 && !accumulate && big_fwd_ok(dtype, N, D, H, W, c0, c1) &&
      (long)N * D * H * W * Cout * 2 < (long)kOOB) {
    p.nbd = D / kBgBD; p.nbh = H / 8; p.nbw = W / 16;
    const long nvox = (long)N * D * H * W;
    const int nslot = big_slots(N, D, H, W, Cout);
    auto kern = p.isc ? conv3_fwd_big_kernel<true> : conv3_fwd_big_kernel<false>;
    const int ldsb = p.isc ? kBgLdsBn : kBgLds;
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, ldsb);
    hipLaunchKernelGGL(kern, dim3(nslot * (Cout / 64)), dim3(kBgThreads), ldsb, s, p,
                       (uint32_t)(nvox * c0 * 2), (uint32_t)(nvox * c1 * 2));
    PCMS_CHECK_LAUNCH();
  }
  if (p.isc) return -5;  // the input BatchNorm + ReLU runs on the big-box path only
  dim3 grid(N * p.nbd * p.nbh * p.nbw * (Cout / 64) * splits);
  const bool hot = b.lbd == 2 && b.lbh == 3 && b.lbw == 4;
  const bool small = b.lbd + b.lbh + b.lbw <= 8 && g_conv_mtw2;  // <= 256 voxels: 2 M-tiles per wave
  if (dtype == PCMS_BF16) {
    if (hot) hipLaunchKernelGGL((conv3_fwd_kernel<bf16_t, 2, 2, 3, 4>), grid, dim3(kThreads), 0, s, p);
    else if (small) hipLaunchKernelGGL((conv3_fwd_kernel<bf16_t, 2, -1, -1, -1, 2>), grid, dim3(kThreads), 0, s, p);
    else hipLaunchKernelGGL((conv3_fwd_kernel<bf16_t, 2, -1, -1, -1>), grid, dim3(kThreads), 0, s, p);
  } else if (dtype == PCMS_F32X3) {
    if (hot) hipLaunchKernelGGL((conv3_fwd_kernel<x3_t, 2, 2, 3, 4>), grid, dim3(kThreads), 0, s, p);
    else hipLaunchKernelGGL((conv3_fwd_kernel<x3_t, 2, -1, -1, -1>), grid, dim3(kThreads), 0, s, p);
  } else {
    if (hot) hipLaunchKernelGGL((conv3_fwd_kernel<x6_t, 2, 2, 3, 4>), grid, dim3(kThreads), 0, s, p);
    else if (small) hipLaunchKernelGGL((conv3_fwd_kernel<x6_t, 2, -1, -1, -1, 2>), grid, dim3(kThreads), 0, s, p);
    else hipLaunchKernelGGL((conv3_fwd_kernel<x6_t, 2, -1, -1, -1>), grid, dim3(kThreads), 0, s, p);
  }
  PCMS_CHECK_LAUNCH();
}

extern "C" {



// Weight-gradient launch plan: box geometry, boxes per split, split count (shared by the
// launch and its workspace query)
// bf16 grids of at most this many boxes split their taps over two workgroups (TG) before
// splitting their voxels (partial rows + a reduction pass); 0 disables
static int g_wgrad_tg_maxbox = 64;
// compile-time-box bf16 weight gradients on v_mfma_f32_16x16x32_bf16 (1) or 32x32x16 (0, the
// product: the 16x16x32 form ran at a higher clock but slower, profiles/r5_wgrad_k16_abl.txt)
static int g_wgrad_k16 = 0;
// the fp32 build's weight gradient streams its boxes by LDS-DMA into an fp32 staging buffer (1)
// or stages each box synchronously through registers (0, the product): with the 64-voxel boxes
// of round 6 both run the fp32 step in the same time (66.5 vs 66.2 ms, profiles/r6_x6_ab.txt) --
// the kernel is bound by its LDS fragment reads, not by the box stream
static int g_wgrad_x6_dma = 0;
struct WgradPlan { Box b; int nbd, nbh, nbw, nbox, bps, splits, ntg; };
static WgradPlan wgrad_plan(int dtype, int N, int D, int H, int W, int Cin, int Cout, int target_wgs) {
  WgradPlan q;
  const int bv = dtype == PCMS_BF16 ? WTraits<bf16_t>::BV : dtype == PCMS_F32X3 ? WTraits<x3_t>::BV : WTraits<x6_t>::BV;
  const int halo = dtype == PCMS_F32 ? WTraits<x6_t>::HALO : kWHaloMax;
  q.b = choose_box(D, H, W, bv, halo, 4, 16);
  q.nbd = cdiv(D, 1 << q.b.lbd); q.nbh = cdiv(H, 1 << q.b.lbh); q.nbw = cdiv(W, 1 << q.b.lbw);
  q.nbox = N * q.nbd * q.nbh * q.nbw;
  const int tiles = (Cout / 64) * cdiv(Cin, 32);
  if (target_wgs <= 0) target_wgs = 512;
  q.ntg = dtype == PCMS_BF16 && q.nbox <= g_wgrad_tg_maxbox && tiles < target_wgs ? 2 : 1;
  const int splits = std::max(1, std::min(q.nbox, cdiv(target_wgs, tiles * q.ntg)));
  q.bps = cdiv(q.nbox, splits);
  q.splits = cdiv(q.nbox, q.bps);
  return q;
}

// the compile-time-box bf16 weight gradients on 16x16x32 (1) or 32x32x16 (0) MFMAs; v < 0
// queries.  Returns the previous value.
int pcms_conv3_wgrad_k16(int v) {
  const int old = g_wgrad_k16;
  if (v >= 0) g_wgrad_k16 = v;
  return old;
}

// the fp32 (bf16x6) weight gradient's LDS-DMA box stream (1) or synchronous staging (0); v < 0
// queries.  Returns the previous value.
int pcms_conv3_wgrad_x6_dma(int v) {
  const int old = g_wgrad_x6_dma;
  if (v >= 0) g_wgrad_x6_dma = v;
  return old;
}

// the weight gradient's split rows summed by one launch (1) or by the two-stage group-sum +
// reduce pair (0), bit-identical; v < 0 queries.  Returns the previous value.
int pcms_conv3_wgrad_reduce_fused(int v) {
  const int old = g_wred_fused;
  if (v >= 0) g_wred_fused = v;
  return old;
}

// grids of at most v boxes split the taps of the bf16 weight gradient over two workgroups
// before splitting the voxels (0: never); v < 0 queries.  Returns the previous value.
int pcms_conv3_wgrad_tg_maxbox(int v) {
  const int old = g_wgrad_tg_maxbox;
  if (v >= 0) g_wgrad_tg_maxbox = v;
  return old;
}

// fp32 workspace floats pcms_conv3_wgrad needs: one [27][Cout][c0+c1] partial row per split
int pcms_conv3_wgrad_ws_floats(int dtype, int N, int D, int H, int W, int c0, int c1, int Cout, int target_wgs) {
  const int Cin = c0 + c1;
  return wgrad_plan(dtype, N, D, H, W, Cin, Cout, target_wgs).splits * 27 * Cout * Cin;
}

// Weight gradient: dw (torch layout [Cout][cin_w][27], fp32) += sum_v dy (x) x, where
// cin_w <= c0 + c1 is the weight's input-channel count (the stored input may be padded).
// dwt: pcms_conv3_wgrad_ws_floats(...) fp32 workspace (per-split partial rows, summed in a
// fixed order: the result is deterministic).
static int conv3_wgrad_any(int dtype, const void* x0, int c0, const void* x1, int c1, const float* isc,
                           const float* ish, const void* dy, float* dw, float* dwt, int N, int D, int H, int W,
                           int Cout, int cin_w, int target_wgs, int flags, hipStream_t s);

int pcms_conv3_wgrad(int dtype, const void* x0, int c0, const void* x1, int c1, const void* dy,
                     float* dw, float* dwt, int N, int D, int H, int W, int Cout, int cin_w, int target_wgs,
                     int flags, hipStream_t s) {
  return conv3_wgrad_any(dtype, x0, c0, x1, c1, nullptr, nullptr, dy, dw, dwt, N, D, H, W, Cout, cin_w, target_wgs,
                         flags, s);
}

// 1: pcms_conv3_fwd_bnin and pcms_conv3_wgrad_bnin (target_wgs) both run this bf16 layer
int pcms_conv3_bnin_ok(int N, int D, int H, int W, int cin, int Cout, int target_wgs) {
  const long nvox = (long)N * D * H * W;
  if (cin > kBgBnMax || cin % 16 || Cout % 64 || !big_fwd_ok(PCMS_BF16, N, D, H, W, cin, 0)) return 0;
  if (nvox * std::max(Cout, cin) * 2 >= (long)kOOB) return 0;
  return wgrad_plan(PCMS_BF16, N, D, H, W, cin, Cout, target_wgs).ntg == 1 ? 1 : 0;
}

// the weight gradient of the conv of relu(x * isc + ish) (pcms_conv3_fwd_bnin's forward):
// bf16, one source; the LDS-DMA shapes only (-5 otherwise)
int pcms_conv3_wgrad_bnin(int dtype, const void* x, int cin, const float* isc, const float* ish, const void* dy,
                          float* dw, float* dwt, int N, int D, int H, int W, int Cout, int cin_w, int target_wgs,
                          int flags, hipStream_t s) {
  if (!isc || !ish || dtype != PCMS_BF16) return -1;
  return conv3_wgrad_any(dtype, x, cin, nullptr, 0, isc, ish, dy, dw, dwt, N, D, H, W, Cout, cin_w, target_wgs,
                         flags, s);
}

}  // extern "C"

static int conv3_wgrad_any(int dtype, const void* x0, int c0, const void* x1, int c1, const float* isc,
                           const float* ish, const void* dy, float* dw, float* dwt, int N, int D, int H, int W,
                           int Cout, int cin_w, int target_wgs, int flags, hipStream_t s) {
  const int Cin = c0 + c1;
  if (cin_w <= 0 || cin_w > Cin) return -4;
  if (flags & ~PCMS_GRAD_STORE) return -8;
  const int VEC = dtype == PCMS_BF16 ? 8 : 4;
  if (Cout % 64 != 0 || c0 % VEC != 0 || c1 % VEC != 0) return -1;
  const WgradPlan q = wgrad_plan(dtype, N, D, H, W, Cin, Cout, target_wgs);
  WgradParams p;
  p.x0 = x0; p.x1 = x1; p.c0 = c0; p.c1 = c1; p.dy = dy; p.dwt = dwt;
  p.N = N; p.D = D; p.H = H; p.W = W; p.Cin = Cin; p.Cout = Cout;
  p.lbd = q.b.lbd; p.lbh = q.b.lbh; p.lbw = q.b.lbw;
  p.nbd = q.nbd; p.nbh = q.nbh; p.nbw = q.nbw;
  p.nbox = q.nbox;
  p.boxes_per_split = q.bps;
  const long nvox = (long)N * D * H * W;
  // LDS-DMA staging: bf16, and the fp32 (bf16x6) build's fp32 staging buffer (g_wgrad_x6_dma)
  const int es = dtype == PCMS_BF16 ? 2 : 4;
  p.dma = (dtype == PCMS_BF16 || (dtype == PCMS_F32 && g_wgrad_x6_dma)) && (c1 == 0 || c0 % 32 == 0) &&
          nvox * std::max(Cout, std::max(c0, c1)) * es < (long)kOOB;
  p.x0bytes = (uint32_t)(p.dma ? nvox * c0 * es : 0);
  p.x1bytes = (uint32_t)(p.dma ? nvox * c1 * es : 0);
  p.dybytes = (uint32_t)(p.dma ? nvox * Cout * es : 0);
  const int splits = q.splits;
  p.nco = Cout / 64;
  p.nci = cdiv(Cin, 32);
  p.dw = dw;
  p.cw = cin_w;
  p.direct = splits == 1;
  p.store = flags & PCMS_GRAD_STORE;
  p.ntg = q.ntg;
  p.isc = isc; p.ish = ish;
  if (isc && (!p.dma || c1 != 0 || q.ntg != 1)) return -5;  // BNIN: the LDS-DMA one-source kernels
  dim3 grid(splits * p.nco * p.nci * q.ntg);
  size_t lds;
  if (dtype == PCMS_BF16 && isc) {
    lds = (size_t)WTraits<bf16_t>::NBUF * (WTraits<bf16_t>::BV * WTraits<bf16_t>::DYROW + kWHaloMax * WTraits<bf16_t>::XROW) +
          64 * sizeof(float);
    auto kern = conv3_wgrad_kernel<bf16_t, -1, -1, -1, false, false, true>;
    const bool k16 = g_wgrad_k16;
    if (q.b.lbd == 2 && q.b.lbh == 2 && q.b.lbw == 4)
      kern = k16 ? conv3_wgrad_kernel<bf16_t, 2, 2, 4, false, false, true, true> : conv3_wgrad_kernel<bf16_t, 2, 2, 4, false, false, true>;
    else if (q.b.lbd == 1 && q.b.lbh == 3 && q.b.lbw == 4)
      kern = k16 ? conv3_wgrad_kernel<bf16_t, 1, 3, 4, false, false, true, true> : conv3_wgrad_kernel<bf16_t, 1, 3, 4, false, false, true>;
    else if (q.b.lbd == 2 && q.b.lbh == 3 && q.b.lbw == 3)
      kern = k16 ? conv3_wgrad_kernel<bf16_t, 2, 3, 3, false, false, true, true> : conv3_wgrad_kernel<bf16_t, 2, 3, 3, false, false, true>;
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(kern, grid, dim3(kWThreads), lds, s, p);
  } else if (dtype == PCMS_BF16) {
    lds = (size_t)WTraits<bf16_t>::NBUF * (WTraits<bf16_t>::BV * WTraits<bf16_t>::DYROW + kWHaloMax * WTraits<bf16_t>::XROW);
    auto kern = conv3_wgrad_kernel<bf16_t, -1, -1, -1>;
    if (q.ntg == 2) {
      kern = conv3_wgrad_kernel<bf16_t, -1, -1, -1, true>;
      if (q.b.lbd == 2 && q.b.lbh == 3 && q.b.lbw == 3) kern = conv3_wgrad_kernel<bf16_t, 2, 3, 3, true>;
    } else if (q.b.lbd == 2 && q.b.lbh == 2 && q.b.lbw == 4) {
      kern = g_wgrad_k16 ? conv3_wgrad_kernel<bf16_t, 2, 2, 4, false, false, false, true> : conv3_wgrad_kernel<bf16_t, 2, 2, 4>;
    } else if (q.b.lbd == 1 && q.b.lbh == 3 && q.b.lbw == 4) {
      kern = g_wgrad_k16 ? conv3_wgrad_kernel<bf16_t, 1, 3, 4, false, false, false, true> : conv3_wgrad_kernel<bf16_t, 1, 3, 4>;
    } else if (q.b.lbd == 2 && q.b.lbh == 3 && q.b.lbw == 3) {
      kern = g_wgrad_k16 ? conv3_wgrad_kernel<bf16_t, 2, 3, 3, false, false, false, true> : conv3_wgrad_kernel<bf16_t, 2, 3, 3>;
    } else if (q.b.lbd == 3 && q.b.lbh == 3 && q.b.lbw == 2) {  // level 4
      kern = g_wgrad_k16 ? conv3_wgrad_kernel<bf16_t, 3, 3, 2, false, false, false, true> : conv3_wgrad_kernel<bf16_t, 3, 3, 2>;
    }
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(kern, grid, dim3(kWThreads), lds, s, p);
  } else if (dtype == PCMS_F32X3) {
    typedef WTraits<x3_t> X;
    lds = (size_t)X::NPART * (X::BV * X::DYROW + X::HALO * X::XROW);
    (void)hipFuncSetAttribute((const void*)conv3_wgrad_kernel<x3_t, -1, -1, -1>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL((conv3_wgrad_kernel<x3_t, -1, -1, -1>), grid, dim3(kWThreads), lds, s, p);
  } else {
    typedef WTraits<x6_t> X;
    lds = (size_t)X::NPART * (X::BV * X::DYROW + X::HALO * X::XROW) + (p.dma ? X::RAWBYTES : 0);
    // the direct (one-split) flush transposes a [32 co][32 ci][27] fp32 tile through LDS
    if (p.direct) lds = std::max(lds, (size_t)32 * 32 * 27 * sizeof(float));
    auto kern = Cin <= 8 ? conv3_wgrad_kernel<x6_t, -1, -1, -1, false, true> : conv3_wgrad_kernel<x6_t, -1, -1, -1>;
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(kern, grid, dim3(kWThreads), lds, s, p);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  if (p.direct) return 0;  // the kernel added into dw itself
  const long E = 27L * Cout * Cin;
  const int G = cdiv(splits, 16);
  if (g_wred_fused && G <= kWredMaxGroups && E * 16 * 4 < (1L << 31)) {
    const dim3 grid(Cout, cdiv(cin_w, 32));
    const size_t glds = (size_t)G * 27 * 32 * sizeof(float);
    if (G >= 4)
      hipLaunchKernelGGL(wgrad_reduce_fused_kernel<4>, grid, dim3(1024), glds, s, (const float*)dwt, splits, dw, Cout,
                         Cin, cin_w, p.store);
    else if (G >= 2)
      hipLaunchKernelGGL(wgrad_reduce_fused_kernel<2>, grid, dim3(512), glds, s, (const float*)dwt, splits, dw, Cout,
                         Cin, cin_w, p.store);
    else
      hipLaunchKernelGGL(wgrad_reduce_fused_kernel<1>, grid, dim3(256), glds, s, (const float*)dwt, splits, dw, Cout,
                         Cin, cin_w, p.store);
    PCMS_CHECK_LAUNCH();
  }
  int R = splits, stride = 1;
  if (splits > 16) {
    hipLaunchKernelGGL(wgrad_group_sum_kernel, dim3((unsigned)cdiv(E, 256), cdiv(splits, 16)), dim3(256), 0, s, dwt,
                       splits, E);
    e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
    R = cdiv(splits, 16);
    stride = 16;
  }
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(Cout, cdiv(cin_w, 32)), dim3(256), 0, s, (const float*)dwt, R, stride,
                     dw, Cout, Cin, cin_w, p.store);
  PCMS_CHECK_LAUNCH();
}
