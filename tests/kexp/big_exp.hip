// Big-box forward experiments (test tooling only): the product kernel with parts switched
// off, to see which part bounds the chunk loop.  F bits: 1 halo DMA reads nothing (the
// instructions still issue), 2 B loads all hit one L1 line, 4 no output stores, 8 no A
// fragment reads after the first tap, 16 no MFMAs.
#include "../../prostate-cancer-multimodal-segmentation_amd/csrc/conv3.hip"
namespace {
template <int F>
__global__ void __launch_bounds__(kBgThreads, 1) big_exp_kernel(Conv3Params p, uint32_t x0bytes,
                                                                     uint32_t x1bytes) {
  constexpr int MT = kBgMT;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r_lane = lane & 31, hsel = lane >> 5;
  const int Cout = p.Cout, ncob = Cout >> 6;
  // logical workgroup id: consecutive ids on one XCD (dispatch is round-robin over 8), output
  // channel block fastest, so the workgroups sharing a halo (and neighbouring boxes) share L2
  const int G = gridDim.x;
  const int lg = (G & 7) == 0 ? (blockIdx.x & 7) * (G >> 3) + (blockIdx.x >> 3) : blockIdx.x;
  const int cob = lg % ncob, slot = lg / ncob, nslot = G / ncob;
  const int nbox = p.N * p.nbd * p.nbh * p.nbw;
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
    if (!(F & 1) && live && hv < kBgHalo && (unsigned)gd < (unsigned)p.D && (unsigned)gh < (unsigned)p.H &&
        (unsigned)gw < (unsigned)p.W)
      voff = ((uint32_t)(((n * p.D + gd) * p.H + gh) * p.W + gw) * stride + cofs +
              (uint32_t)((pc & 1) ^ ((hw_ >> 3) & 1)) * 8u) * 2u;
    if constexpr ((F & 32) != 0) voff = voff == kOOB ? kOOB : (voff & 0xFFFFFu);  // halo from 1 MiB (L2-resident)
    // contiguous pieces (what a 16-channel-blocked layout would fetch: every wave
    // instruction one 1 KiB run), same byte count and LDS placement, wrong data
    if constexpr ((F & 128) != 0)
      voff = voff == kOOB ? kOOB : (((uint32_t)((n * p.D + d0) * p.H + h0) * 1024u + (uint32_t)pc * 16u + (uint32_t)chunk * 4096u) % (x0bytes - 16u)) & ~15u;
    const uint32_t lb = __builtin_amdgcn_readfirstlane(lds0 + buf * kBgBuf + (wave * 64 + j * kBgThreads) * 16);
    dma16(first ? xr0 : xr1, lb, voff, 0);
  };

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
  auto load_b = [&](s16x8_t (&dst)[2], int chunk, int tap, uint32_t boff) {
    const uint32_t off = (F & 2) ? boff : boff + (uint32_t)((chunk >> 1) * 27 + tap) * tap_bytes + (uint32_t)(chunk & 1) * 32u;
    bload16<0>(dst[0], wr, off);
    bload16<64>(dst[1], wr, off);
  };

  // epilogue constants: output columns are channel pairs (column j of N-tile nt = channel
  // 2 j + nt); two-pointer output split at cy0 (workgroup-uniform)
  // (bias and the running BatchNorm moments live in LDS between boxes, not in registers)
  float* red = reinterpret_cast<float*>(lds + 2 * kBgBuf + 4 * kBgStage);  // [wave][64][3]
  float* bls = red + 4 * 64 * 3;                                           // [64]
  if (tid < 64) bls[tid] = p.bias ? p.bias[co_base + tid] : 0.f;
  const bool to0 = co_base < p.cy0;
  const long ys = to0 ? p.cy0 : Cout - p.cy0;
  const int yc0 = to0 ? co_base : co_base - p.cy0;
  // output through a descriptor too (stores out of range are dropped; the host checks
  // every byte offset fits 31 bits)
  const __amdgpu_buffer_rsrc_t yr = __builtin_amdgcn_make_buffer_rsrc(
      to0 ? p.y0 : p.y1, (short)0, (int)(p.nvox * ys * 2), 0x00020000);
  char* stg = lds + 2 * kBgBuf + wave * kBgStage;
  int nbdone = 0;  // boxes merged into the running moments (uniform: kept in an SGPR)

  f32x16_t acc[MT][2];
  s16x8_t bset[kBgDist + 1][2];
  int box = slot;
  int n, d0, h0, w0;
  origin(box, n, d0, h0, w0);
  if constexpr ((F & 64) != 0) {
    // desynchronise: odd slots start ~half a box later (store bursts of neighbouring CUs
    // no longer coincide)
    // p.accumulate = (modulus << 8) | sleeps per step: slot s waits (s % modulus) * sleeps
    const int mod = p.accumulate >> 8, units = p.accumulate & 255;
    const int k = mod > 0 ? (slot % mod) * units : 0;
    for (int i = 0; i < k; ++i) __builtin_amdgcn_s_sleep(127);
  }
#pragma unroll
  for (int j = 0; j < kBgPieces; ++j) stage_piece(n, d0, h0, w0, 0, 0, j, true);
#pragma unroll
  for (int t = 0; t < kBgDist; ++t) load_b(bset[t], 0, t, (uint32_t)((co_base + 2 * r_lane) * 64 + hsel * 16));
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int buf = 0;
  while (true) {
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
    const int nbx = box + nslot;
    const bool has_next = nbx < nbox;
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
      const int hbase = ((2 * wave * kBgHH + (prow >> 4)) * kBgHW + (prow & 15)) * 32;
      int swk[3];
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) swk[kw] = hbase + kw * 32 + ((hs ^ ((((prow & 15) + kw) >> 3) & 1)) << 4);
      const uint32_t boff = (uint32_t)((co_base + 2 * (lo & 31)) * 64 + hs * 16);
      auto read_a1 = [&](int tap, int mt) {
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
        if constexpr (tap < kBgPieces) stage_piece(sn, sd, sh, sw, schunk, buf ^ 1, tap, live);
        s16x8_t(&b)[2] = bset[tap % (kBgDist + 1)];
        constexpr int extra = (Slack && tap < kBgDist) ? kBgEpiStores : 0;
        vm_wait2<bg_wait<kBgPieces, kBgDist>(tap) + extra>(b[0], b[1]);
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
          if constexpr (!(F & 16)) {
            acc[mt][0] = mfma(a[mt], b[0], acc[mt][0]);
            acc[mt][1] = mfma(a[mt], b[1], acc[mt][1]);
          } else {
            acc[mt][0][0] += (float)a[mt][0] * (float)b[0][0];
            acc[mt][1][0] += (float)a[mt][1] * (float)b[1][0];
          }
          if constexpr (tap + 1 < 27 && !(F & 8)) a[mt] = read_a1(tap + 1, mt);
        }
      });
      // the next chunk's halo has landed (the newest piece is followed by the B loads of the
      // remaining taps) and every wave is done with buf.  After a box's last chunk retire
      // everything: the epilogue needs registers, and the compiler may move (or, after the
      // workgroup's last box, reuse) the destinations of the next box's B loads -- they
      // must hold landed data by then (costs one L2 round trip per box).
      if (!last) vm_wait<2 * (27 - kBgPieces)>();
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      buf ^= 1;
    };
    run_chunk(0, std::true_type{});
    for (int chunk = 1; chunk < nchunk; ++chunk) run_chunk(chunk, std::false_type{});

    // ---- epilogue of this box, two M-tiles at a time: + bias, bf16 pairs into the wave's
    // LDS slice (row = 32 mm + C row, 128 B of 32 channel pairs), read back as 8 x 16 B per
    // lane = whole 128-B channel rows, 16-B stores.  BatchNorm moments in the same pass,
    // shifted by K (the running mean; the bias before the first box): box mean K + S1 / n,
    // M2 = S2 - S1^2 / n, Chan-merged into the running moments.
    // (lane-dependent offsets from an opaque lane copy: box-invariant, the compiler would
    // hoist them out of the box loop and spill them)
    const int lane_o = opaque(lane);
    const long plane = (long)p.H * p.W;
    const long vbase = (((long)n * p.D + d0) * p.H + h0) * p.W + w0;
    char* wst = stg + (lane_o & 31) * 4 + (lane_o >> 5) * 512;
    float* rme = red + (wave * 64 + 2 * (lane_o & 31)) * 3;  // [ch][mean, M2, n] x 2 channels
    const float bias0 = bls[2 * (lane_o & 31)], bias1 = bls[2 * (lane_o & 31) + 1];
    const float rn = (float)nbdone * (32.f * MT);
    const float K0 = nbdone ? rme[0] : bias0, K1 = nbdone ? rme[3] : bias1;
    const float c0s = bias0 - K0, c1s = bias1 - K1;  // d = acc + bias - K
    float S1[2] = {0.f, 0.f}, S2[2] = {0.f, 0.f};
#pragma unroll
    for (int pass = 0; pass < MT / 2; ++pass) {
#pragma unroll
      for (int mm = 0; mm < 2; ++mm)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int row = mm * 32 + (e & 3) + 8 * (e >> 2);
          const float v0 = acc[2 * pass + mm][0][e], v1 = acc[2 * pass + mm][1][e];
          *reinterpret_cast<uint32_t*>(wst + row * 128) = pack_bf16x2(v0 + bias0, v1 + bias1);
          const float e0 = v0 + c0s, e1 = v1 + c1s;
          S1[0] += e0;
          S1[1] += e1;
          S2[0] = fmaf(e0, e0, S2[0]);
          S2[1] = fmaf(e1, e1, S2[1]);
        }
      asm volatile("" ::: "memory");
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int row = k * 8 + (lane_o >> 3), c16 = lane_o & 7;
        const u32x4_t v = *reinterpret_cast<const u32x4_t*>(stg + row * 128 + c16 * 16);
        const int mt = 2 * pass + (row >> 5), pr = perm32(row & 31);
        const int rd = 2 * wave + (mt >> 2), rh = 2 * (mt & 3) + (pr >> 4), rw = pr & 15;
        const long vox = vbase + (long)rd * plane + (long)rh * p.W + rw;
        if constexpr (!(F & 4))
          __builtin_amdgcn_raw_buffer_store_b128(v, yr, (int)((vox * ys + yc0 + c16 * 8) * 2), 0,
                                                 (F & 256) ? 16 : (F & 512) ? 2 : 0);
        else if (v[0] == 0x12345678u && v[1] == 0x9abcdef0u) __builtin_amdgcn_raw_buffer_store_b128(v, yr, 0, 0, 0);
      }
      asm volatile("" ::: "memory");
    }
    {
      constexpr float nb = 32.f * MT;  // voxels per wave and box
      const float nnew = rn + nb;
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        const float s1 = S1[nt] + __shfl_xor(S1[nt], 32, 64);
        const float s2 = S2[nt] + __shfl_xor(S2[nt], 32, 64);
        const float K = nt ? K1 : K0;
        const float mbox = K + s1 / nb;
        const float m2b = fmaxf(s2 - s1 * s1 / nb, 0.f);
        const float rmean = nbdone ? rme[3 * nt] : 0.f, rm2 = nbdone ? rme[3 * nt + 1] : 0.f;
        const float delta = mbox - rmean;
        if ((lane_o >> 5) == 0) {
          rme[3 * nt] = rmean + delta * (nb / nnew);
          rme[3 * nt + 1] = rm2 + m2b + delta * delta * (rn * nb / nnew);
          rme[3 * nt + 2] = nnew;
        }
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

}  // namespace
extern "C" int exp_big(int F, const void* x0, int c0, const void* x1, int c1, const void* w, const float* bias,
                       void* y, float* stats, int N, int D, int H, int W, int Cout, int wgs, hipStream_t s) {
  Conv3Params p = {};
  p.accumulate = wgs >> 16;  // delay config (F & 64)
  wgs &= 0xffff;
  p.x0 = x0; p.x1 = x1; p.c0 = c0; p.c1 = c1; p.w = w; p.bias = bias; p.y0 = y; p.y1 = nullptr; p.cy0 = Cout;
  p.stats = stats; p.N = N; p.D = D; p.H = H; p.W = W; p.Cin = c0 + c1; p.Cout = Cout;
  p.nvox = (long)N * D * H * W;
  p.nbd = D / 8; p.nbh = H / 8; p.nbw = W / 16;
  const int nbox = N * p.nbd * p.nbh * p.nbw;
  const int G = wgs > 0 ? wgs : 256;
  const int nslot = std::min(nbox, G / (Cout / 64));
  auto launch = [&](auto kern) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, kBgLds);
    hipLaunchKernelGGL(kern, dim3(nslot * (Cout / 64)), dim3(kBgThreads), kBgLds, s, p,
                       (uint32_t)(p.nvox * c0 * 2), (uint32_t)(p.nvox * c1 * 2));
  };
  switch (F) {
    case 0: launch(big_exp_kernel<0>); break;
    case 1: launch(big_exp_kernel<1>); break;
    case 2: launch(big_exp_kernel<2>); break;
    case 3: launch(big_exp_kernel<3>); break;
    case 4: launch(big_exp_kernel<4>); break;
    case 7: launch(big_exp_kernel<7>); break;
    case 8: launch(big_exp_kernel<8>); break;
    case 15: launch(big_exp_kernel<15>); break;
    case 16: launch(big_exp_kernel<16>); break;
    case 23: launch(big_exp_kernel<23>); break;
    case 32: launch(big_exp_kernel<32>); break;
    case 36: launch(big_exp_kernel<36>); break;
    case 64: launch(big_exp_kernel<64>); break;
    case 128: launch(big_exp_kernel<128>); break;
    case 256: launch(big_exp_kernel<256>); break;
    case 512: launch(big_exp_kernel<512>); break;
    case 132: launch(big_exp_kernel<132>); break;
    case 68: launch(big_exp_kernel<68>); break;
    default: return -1;
  }
  return (int)hipGetLastError();
}
