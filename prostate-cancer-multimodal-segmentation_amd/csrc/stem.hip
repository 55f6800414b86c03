// Stem convolution (inc.conv.0: n_modalities -> 64, k3 p1), bf16, gfx950: the HBM-bound
// layer of the U-Net (models/unet3d.py:29 inside inc = DoubleConv3D(n_modalities, 64)).
#include "conv_common.h"
#include "pcms_hip.h"

namespace {

// ------------------------------------------------------------------------------------
// Stem conv (inc.conv.0: n_modalities -> 64, input stored with 8 channels), bf16.
// The generic kernel would spend 4x its MFMA work on zero channels (K = 27 x 32); here the
// K dimension packs two taps per MFMA k-step: k = (tap 2s + h, channel c), h = lane >> 5,
// so K = 14 x 16 = 224 (135 real).  HBM-bound: 16 B in + 128 B out per voxel.
// ------------------------------------------------------------------------------------
constexpr int kStemSteps = 14;                    // 28 taps (27 + 1 zero) / 2
// K-dense form (<= 5 input channels): one k-step per (kd, kh) tap row, k = the three kw taps'
// 5 channels (15 + 1 zero): K = 9 x 16 = 144 (135 real) instead of 224
constexpr int kStemDSteps = 9;
constexpr int kStemPackElems = (kStemSteps + kStemDSteps) * 64 * 16;  // both forms, tap-pair first

// timeline instrumentation hook for tests/kexp (empty in the product library)
#ifndef STEM_STAMP
#define STEM_STAMP(k)
#define STEM_STAMP_END()
#endif

// master W[64][cin_w][27] fp32 -> [14][64][16] bf16, k = h * 8 + c <-> (tap 2s + h, c);
// the 64 output columns are ordered (nt, j) -> channel 2 j + nt so that a lane's two MFMA
// tiles hold an adjacent channel pair (one packed bf16x2 LDS write per row)
// followed by the K-dense form [9][64][16]: step s = tap row (kd, kh) = (s / 3, s % 3), k =
// 5 kw + c for kw < 3, c < 5 (k = 15: zero) -- the order of the R1 | R2 halo windows of
// stem_fwd_direct_kernel<.., DENSE>; zero unless cin_w <= 5
__global__ void stem_pack_kernel(const float* w, bf16_t* out, int cin_w) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= kStemPackElems) return;
  const int k = i & 15, col = (i >> 4) & 63, s = i >> 10;
  const int co = 2 * (col & 31) + (col >> 5);  // MFMA column (nt, j) <-> channel 2 j + nt
  float v = 0.f;
  if (s < kStemSteps) {
    const int tap = 2 * s + (k >> 3), c = k & 7;
    if (tap < 27 && c < cin_w) v = w[((long)co * cin_w + c) * 27 + tap];
  } else {
    const int sd = s - kStemSteps, kw = k / 5, c = k % 5;
    if (k < 15 && c < cin_w && cin_w <= 5) v = w[((long)co * cin_w + c) * 27 + sd * 3 + kw];
  }
  out[i] = f2bf(v);
}

__device__ __forceinline__ int tap_off(int tap, int HH, int HW) {
  if (tap >= 27) return 0;  // zero-weight pad tap: any in-halo row
  const int kd = tap / 9, kh = (tap / 3) % 3, kw = tap % 3;
  return (kd * HH + kh) * HW + kw;
}

// Persistent stem forward for 16-wide 512-voxel boxes (bd x bh = 32): one 8-wave workgroup
// per CU walks boxes b = blockIdx.x + k gridDim.x; wave w computes the 64 voxels [64 w, 64 w
// + 64) of each box (2 M-tiles x 2 N-tiles of v_mfma_f32_32x32x16_bf16, K = 14 tap-pair steps).
//  * Stores: the weight columns are ordered so that lane r_lane holds channels (2 r_lane,
//    2 r_lane + 1) of its rows, so the 32 lanes of a half-wave write one voxel's 64 channels
//    (128 contiguous bytes) with ONE buffer_store_dword (per-lane voffset, wave-uniform
//    soffset, immediate offset: no VALU address math, no LDS round trip).
//  * Halo: double-buffered, buffer LDS-DMA (out-of-range voffset = zero padding), the next
//    box's halo in flight while this one computes; one raw barrier per box (the stores of
//    a box stay in flight across it: vmcnt counts loads, stores and DMA in issue order).
//  * Weights: in LDS (28 KiB, k-halves swapped on column bit 4: conflict-free reads).
//  * Staggered epilogue: waves 0-3 do each box's epilogue (BN sums, bf16 packing, stores)
//    right after its MFMAs; waves 4-7 defer theirs to the start of the NEXT box, so on every
//    SIMD one wave's MFMAs run beside the other wave's vector / store work instead of the
//    two waves doing the same phase at once (MFMA and VALU pipes are separate).
//  * BatchNorm partials: shifted sums over all boxes of the workgroup, ONE stats row per
//    workgroup (rows >= gridDim.x are zeroed: count 0).
// halo rows in LDS are padded from 18 to kSDHW = 24 voxels (384 B = 128 B mod 256): the two
// H-rows a 16-lane ds_read_b128 group reads land on disjoint halves of the 256-B bank row
constexpr int kSDHW = 24;
// 1440 halo rows ((bd+2)(bh+2) = 60), rounded up to whole 64-row DMA pieces: a wave's last
// piece writes all 64 of its rows (the ones past the halo get zeros)
constexpr int kSDHaloRows = (6 * 10 * kSDHW + 63) / 64 * 64;
constexpr int kSDHaloBytes = kSDHaloRows * 16;
constexpr int kSDW = 2 * kSDHaloBytes;                        // weights [14][64][32 B]
constexpr int kSDRed = kSDW + kStemSteps * 64 * 32;
constexpr int kSDLds = kSDRed + 8 * 64 * 3 * 4;               // + stats reduction
// K-dense form: the two raw halo buffers, then the repacked windows R (960 rows x 32 B: the
// box's (bd + 2)(bh + 2) tap rows x 16 output w), weights [9][64][32 B], stats reduction
constexpr int kSDRRows = 6 * 10 * 16;
constexpr int kSDRBytes = kSDRRows * 32;
constexpr int kSD2R = 2 * kSDHaloBytes;                       // two R buffers
constexpr int kSD2W = kSD2R + 2 * kSDRBytes;
constexpr int kSD2Red = kSD2W + kStemDSteps * 64 * 32;
constexpr int kSD2Lds = kSD2Red + 8 * 64 * 3 * 4;
static_assert(kSD2Lds <= 160 * 1024, "LDS");
constexpr int kSDThr = 512;                                   // one 8-wave workgroup per CU

// Output stores.  PCMS_STEM_WIDE 1: 16-B stores of whole 128-B voxel rows.  A
// lane holds channels (2 j', 2 j' + 1) of 16 voxels per M-tile (j' = its MFMA column), so the
// four lanes of a quad hold channels 8 k .. 8 k + 7 (k = column >> 2) of the same four
// w-consecutive voxels of a group g; a 4 x 4 transpose inside the quad (two DPP quad_perm
// stages, each lane selecting between its own and its partner's register) leaves lane j of
// the quad with voxel 4 g + j's channels 8 k .. 8 k + 7: one buffer_store_dwordx4 per group
// writes 8 whole voxel rows (1 KiB).  8 store instructions per wave and box instead of 32
// dword stores; the same bytes to the same addresses.  0 (the product): the dword stores --
// A/B on one box, standalone launches: wide 84.4 / 82.9 us vs dword 80.5 / 78.8 us, the
// 16 DPP + select VALU per group cost more than the 24 store instructions they save.
#ifndef PCMS_STEM_WIDE
#define PCMS_STEM_WIDE 0
#endif
// dword stores: the voxel row's constant offset in voffset (folded into the immediate offset
// field, 1) or added to the SGPR soffset (0: an s_add per store)
#ifndef PCMS_STEM_VOFF
#define PCMS_STEM_VOFF 1
#endif

// DPP quad_perm controls: lane j reads lane j ^ 1 / j ^ 2 of its quad
constexpr int kDppXor1 = 0xB1;  // quad_perm [1, 0, 3, 2]
constexpr int kDppXor2 = 0x4E;  // quad_perm [2, 3, 0, 1]
template <int CTRL> __device__ __forceinline__ uint32_t quad_xchg(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xf, 0xf, true);
}
// d[m] of quad lane j = element (j, m) -> element (m, j): lane j ends with d[c] = old d[j] of
// lane c.  Stage s (xor 1, then xor 2) swaps (j, m) with (j ^ s, m ^ s) where bit s of j and
// m differ: for the register pair (m0, m1 = m0 | s), a lane with the bit clear keeps d[m0]
// and takes its partner's d[m0] as d[m1]; with the bit set it keeps d[m1] and takes the
// partner's d[m1] as d[m0].
__device__ __forceinline__ void quad_transpose4(uint32_t (&d)[4], bool b0, bool b1) {
  {
    const uint32_t x0 = quad_xchg<kDppXor1>(d[0]), x1 = quad_xchg<kDppXor1>(d[1]);
    const uint32_t x2 = quad_xchg<kDppXor1>(d[2]), x3 = quad_xchg<kDppXor1>(d[3]);
    const uint32_t n0 = b0 ? x1 : d[0], n1 = b0 ? d[1] : x0;
    const uint32_t n2 = b0 ? x3 : d[2], n3 = b0 ? d[3] : x2;
    d[0] = n0; d[1] = n1; d[2] = n2; d[3] = n3;
  }
  {
    const uint32_t x0 = quad_xchg<kDppXor2>(d[0]), x1 = quad_xchg<kDppXor2>(d[1]);
    const uint32_t x2 = quad_xchg<kDppXor2>(d[2]), x3 = quad_xchg<kDppXor2>(d[3]);
    const uint32_t n0 = b1 ? x2 : d[0], n2 = b1 ? d[2] : x0;
    const uint32_t n1 = b1 ? x3 : d[1], n3 = b1 ? d[3] : x1;
    d[0] = n0; d[1] = n1; d[2] = n2; d[3] = n3;
  }
}

// L2-aware box walk of the persistent stem kernels (boxes are numbered n, d, h, w; w fastest).
// Dispatch is round-robin over the 8 XCDs (workgroup i on XCD i % 8), each with its own 4 MB
// L2, and a box's halo overlaps its d / h / w neighbours' (2 of BD + 2 planes, 2 of BH + 2 rows).
// STEM_WALK 2 (the product): column walk -- every workgroup owns one (n, h, w) box column and
// walks a d range of it (b += nbh nbw), so the 2 halo planes it shares with its previous box
// were staged one step ago by itself; the G / 8 workgroups of one XCD hold consecutive
// columns (h-adjacent), so the halo rows shared across h are staged by a neighbour on the same
// XCD at the same step.  Needs G a multiple of the column count and the d ranges equal;
// otherwise, and for STEM_WALK 1, the XCD-range walk (XCD x walks [x nbox / 8, (x + 1) nbox / 8)
// with its G / 8 workgroups side by side), or the plain b = blockIdx.x + k G (STEM_WALK 0).
#ifndef STEM_WALK
#define STEM_WALK 2
#endif
__device__ inline void stem_box_walk(int nbox, int nbd, int hw, int& b, int& step, int& end) {
  const int G = gridDim.x;
  if (STEM_WALK >= 2 && (G & 7) == 0) {
    const int ncol = nbox / nbd;  // N nbh nbw
    const int sp = G / ncol;      // d ranges per column
    if (sp * ncol == G && nbd % sp == 0) {
      const int lg = (blockIdx.x & 7) * (G >> 3) + (blockIdx.x >> 3);
      const int col = lg % ncol, dr = lg / ncol, dlen = nbd / sp;
      b = ((col / hw) * nbd + dr * dlen) * hw + col % hw;
      step = hw;
      end = b + dlen * hw;
      return;
    }
  }
  if (STEM_WALK >= 1 && (G & 7) == 0 && (nbox & 7) == 0) {
    const int per = nbox >> 3, x = blockIdx.x & 7;
    b = x * per + (blockIdx.x >> 3);
    step = G >> 3;
    end = (x + 1) * per;
  } else {
    b = blockIdx.x;
    step = G;
    end = nbox;
  }
}

// RELU: eval mode with the BatchNorm folded into the weights / bias (the output is the ReLU
// activation; no statistics).
// DENSE (<= 5 input channels, the product): K = 9 tap rows x 16 instead of 14 tap pairs x 16.
// Every thread repacks two of a box's 960 (tap row, w) windows from its landed halo:
// R1 = [x(w) c0-4, x(w + 1) c0-2], R2 = [x(w + 1) c3-4, x(w + 2) c0-4, 0] (halo w), one 32-B
// LDS row per window with the 16-B halves swapped on w bit 3 (a 16-lane read group covers
// all 16 slots of a 256-B bank row); the A fragment of (M-tile, tap row) is then one
// ds_read_b128 of R1 (k-half 0) or R2 (k-half 1), and a box takes 36 MFMAs per wave instead
// of 56.  Pipelined so the repack costs no barrier of its own: the halo DMA runs two boxes
// ahead of the MFMAs and the repack one box ahead, inside the MFMA steps (R double-buffered:
// box b's MFMAs read R[b] while the threads build R[b + 1] from the halo that landed during
// box b - 1; the one barrier per box publishes both).  Measured why it pays: the stem
// forward's MFMA phase does not hide under its store stream (standalone launches, same box:
// 14 MFMA steps 81.3-81.8 us, the first 9 steps only 64.8-67.2 us, none 55.4 us:
// tests/tools/ab_stem_multi.sh with -DSTEM_MFMA_STEPS).
template <int LBD, int LBH, bool RELU, bool DENSE = false>
__global__ void __launch_bounds__(kSDThr, 1) stem_fwd_direct_kernel(Conv3Params p, int nbox, int mrows,
                                                                    uint32_t xbytes, uint32_t ybytes) {
  constexpr int KS = DENSE ? kStemDSteps : kStemSteps;  // MFMA k-steps per box
  constexpr int WOFF = DENSE ? kSD2W : kSDW;
  constexpr int NWV = kSDThr / 64;
  static_assert((1 << (LBD + LBH + 4)) == NWV * 64, "box = 64 voxels per wave");
  constexpr int bd = 1 << LBD, bh = 1 << LBH, bw = 16;
  constexpr int HH = bh + 2, HW = kSDHW, HV = (bd + 2) * HH * HW;  // columns >= bw + 2: zero pad
  constexpr int NP = (HV + kSDThr - 1) / kSDThr;  // halo pieces per thread
  static_assert((HV + 63) / 64 * 64 <= kSDHaloRows, "halo (whole DMA pieces) fits");
  extern __shared__ __attribute__((aligned(16))) char lds[];
  float* red = reinterpret_cast<float*>(lds + (DENSE ? kSD2Red : kSDRed));
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform (SGPR math)
  const int r_lane = lane & 31, hsel = lane >> 5;
  const int D = p.D, H = p.H, W = p.W;
  const i32x4_t xr = buffer_desc(p.x0, xbytes);
  const auto yr = __builtin_amdgcn_make_buffer_rsrc(p.y0, 0, ybytes, 0x00020000);

  // weights -> LDS once (read after the first barrier): row (step, column) of 32 B, its two
  // 16-B k-halves swapped when column bit 3 is set (a 16-lane group then reads 16 distinct
  // 16-B slots of the bank row)
  {
    const u32x4_t* wg = reinterpret_cast<const u32x4_t*>(p.w) + (DENSE ? kStemSteps * 64 * 2 : 0);
    for (int i = tid; i < KS * 64 * 2; i += kSDThr) {
      const int row = i >> 1, half = i & 1, col = row & 63;
      *reinterpret_cast<u32x4_t*>(lds + WOFF + row * 32 + ((half ^ ((col >> 3) & 1)) * 16)) = wg[i];
    }
  }
  const char* wl = lds + WOFF + r_lane * 32 + ((hsel ^ ((r_lane >> 3) & 1)) * 16);
  float bias_l[2] = {0.f, 0.f};
  if (p.bias) { bias_l[0] = p.bias[2 * r_lane]; bias_l[1] = p.bias[2 * r_lane + 1]; }
  // halo rows of the two 32-row MFMA tiles (perm32 layout)
  int hb16[2];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) {
    const int r = wave * 64 + mt * 32 + perm32(r_lane);
    const int rd = r >> (LBH + 4), rh = (r >> 4) & (bh - 1), rw = r & 15;
    if constexpr (DENSE)  // window row (rd, rh, rw) of R buffer 0, k-half hsel
      hb16[mt] = kSD2R + ((rd * HH + rh) * 16 + rw) * 32 + ((((rw >> 3) & 1) ^ hsel) * 16);
    else
      hb16[mt] = ((rd * HH + rh) * HW + rw) * 16;
  }
  static_assert(!DENSE || (bd + 2) * HH * 16 <= kSDRRows, "windows fit R");
  // halo pieces of this thread: relative source offset (bytes) and packed coordinates
  int prel[NP], pco[NP];
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    const int hv = tid + i * kSDThr;
    const int hw_ = hv % HW, t_ = hv / HW, hh_ = t_ % HH, hd_ = t_ / HH;
    prel[i] = (((hd_ - 1) * H + (hh_ - 1)) * W + (hw_ - 1)) * 16;
    pco[i] = (hv < HV && hw_ < bw + 2) ? (hd_ | (hh_ << 8) | (hw_ << 16)) : -1;
  }
  // store voffsets: rows x = perm32((e & 3) + 8 g + 4 hsel) have x & 15 = 4 g + (e & 3) and
  // x >> 4 = (g in {1, 2}) ^ hsel
  const uint32_t vb0 = r_lane * 4, vb1 = r_lane * 4 + (uint32_t)W * 128;
  const uint32_t vA = hsel ? vb1 : vb0;  // g = 0, 3
  const uint32_t vB = hsel ? vb0 : vb1;  // g = 1, 2
  // wide stores: quad lane j writes voxel 4 g + j (w), channels 8 k .. (k = r_lane >> 2)
  const uint32_t wb0 = (r_lane & 3) * 128 + (r_lane >> 2) * 16, wb1 = wb0 + (uint32_t)W * 128;
  const uint32_t wA = hsel ? wb1 : wb0, wB = hsel ? wb0 : wb1;
  const bool qb0 = r_lane & 1, qb1 = (r_lane >> 1) & 1;
  uint32_t qd[4];  // the packed channel pairs of the group being assembled

  auto origin = [&](int b, int& n, int& d0, int& h0, int& w0) {
    const int nbw = p.nbw, nbh = p.nbh, nbd = p.nbd;
    int q = b;
    const int bwi = q % nbw; q /= nbw;
    const int bhi = q % nbh; q /= nbh;
    const int bdi = q % nbd;
    n = q / nbd;
    d0 = bdi * bd; h0 = bhi * bh; w0 = bwi * bw;
  };
  auto stage = [&](int b, int buf) {
    int n, d0, h0, w0;
    origin(b, n, d0, h0, w0);
    const int base16 = ((((n * D + d0) * H + h0) * W) + w0) * 16;
    const bool inner = d0 >= 1 && d0 + bd < D && h0 >= 1 && h0 + bh < H && w0 >= 1 && w0 + bw < W;
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      if (wave * 64 + i * kSDThr >= HV) break;  // whole wave past the halo (uniform)
      uint32_t voff = (uint32_t)(base16 + prel[i]);
      const int c = pco[i];
      if (c < 0) {
        voff = kOOB;
      } else if (!inner) {
        const int gd = d0 + (c & 255) - 1, gh = h0 + ((c >> 8) & 255) - 1, gw = w0 + (c >> 16) - 1;
        if ((unsigned)gd >= (unsigned)D || (unsigned)gh >= (unsigned)H || (unsigned)gw >= (unsigned)W) voff = kOOB;
      }
      dma16(xr, __builtin_amdgcn_readfirstlane(lds_addr(lds) + buf * kSDHaloBytes + (wave * 64 + i * kSDThr) * 16), voff, 0);
    }
  };

  float s1[2] = {0.f, 0.f}, s2[2] = {0.f, 0.f}, K[2] = {0.f, 0.f};
  float cnt = 0.f;
  auto is_full = [&](int bb) {
    int n, d0, h0, w0;
    origin(bb, n, d0, h0, w0);
    return d0 + bd <= D && h0 + bh <= H && w0 + bw <= W;
  };
  // store offsets (wave-uniform) of the two 32-voxel tiles of box bb
  auto tile_so = [&](int bb, uint32_t (&so)[2]) {
    int n, d0, h0, w0;
    origin(bb, n, d0, h0, w0);
    const int bv = ((n * D + d0) * H + h0) * W + w0;
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      const int R0 = wave * 4 + mt * 2;  // even (rd, rh) linear index of the tile
      so[mt] = __builtin_amdgcn_readfirstlane((uint32_t)(bv + ((R0 >> LBH) * H + (R0 & (bh - 1))) * W) * 128u);
    }
  };
  // item (mt, e) of a full box's epilogue: one packed channel-pair store (the 32 lanes of a
  // half-wave write one voxel's 128 B) + the shifted BN sums
  auto item_full = [&](f32x16_t (&acc)[2][2], int mt, int e, const uint32_t (&so)[2]) {
    const int g = e >> 2, rw = 4 * g + (e & 3);
    const float v0 = acc[mt][0][e], v1 = acc[mt][1][e];
    const uint32_t pk = RELU ? pack_bf16x2(fmaxf(v0, 0.f), fmaxf(v1, 0.f)) : pack_bf16x2(v0, v1);
    if constexpr (PCMS_STEM_WIDE) {
      qd[e & 3] = pk;
      if ((e & 3) == 3) {  // the group's four voxels are packed: transpose, one 16-B store
        quad_transpose4(qd, qb0, qb1);
        // soffset 0, the wave-uniform tile offset folded into voffset: a 16-B buffer store
        // with an SGPR soffset gets no wait state before a VALU rewrites its data VGPRs (the
        // compiler models that hazard only without a register soffset), and the store then
        // read partly rewritten data (measured: the second dword of the last quad of every
        // 16-lane row wrong in ~1 % of the stores); with soffset 0 hipcc pads it
        __builtin_amdgcn_raw_buffer_store_b128((u32x4_t){qd[0], qd[1], qd[2], qd[3]}, yr,
                                               ((g == 1 || g == 2) ? wB : wA) + so[mt] + 4 * g * 128, 0, 2);
      }
    } else if constexpr (PCMS_STEM_VOFF) {
      // the voxel's constant row offset rides in the instruction's immediate offset (no s_add
      // per store for a soffset of its own)
      __builtin_amdgcn_raw_buffer_store_b32(pk, yr, ((g == 1 || g == 2) ? vB : vA) + rw * 128, so[mt], 2);
    } else {
      __builtin_amdgcn_raw_buffer_store_b32(pk, yr, (g == 1 || g == 2) ? vB : vA, so[mt] + rw * 128, 2);
    }
    const float e0 = v0 - K[0], e1 = v1 - K[1];
    s1[0] += e0; s2[0] = fmaf(e0, e0, s2[0]);
    s1[1] += e1; s2[1] = fmaf(e1, e1, s2[1]);
  };
  // whole epilogue of one box (boundary boxes, and the last box of the workgroup)
  auto epilogue = [&](f32x16_t (&acc)[2][2], int bb) {
    int n, d0, h0, w0;
    origin(bb, n, d0, h0, w0);
    uint32_t so[2];
    tile_so(bb, so);
    if (is_full(bb)) {
#pragma unroll
      for (int q = 0; q < 32; ++q) item_full(acc, q >> 4, q & 15, so);
      cnt += 32.f;
      return;
    }
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      const int R0 = wave * 4 + mt * 2;
      const int rd0 = R0 >> LBH, rh0 = R0 & (bh - 1);
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int g = e >> 2, rw = 4 * g + (e & 3);
        const bool gB = (g == 1 || g == 2);
        const float v0 = acc[mt][0][e], v1 = acc[mt][1][e];
        const int xh = (gB ? 1 : 0) ^ hsel;
        const bool valid = (d0 + rd0 < D) & (h0 + rh0 + xh < H) & (w0 + rw < W);
        const uint32_t voff = valid ? (gB ? vB : vA) + (PCMS_STEM_VOFF ? rw * 128 : 0) : kOOB;
        const float e0 = valid ? v0 - K[0] : 0.f, e1 = valid ? v1 - K[1] : 0.f;
        cnt += valid ? 1.f : 0.f;
        __builtin_amdgcn_raw_buffer_store_b32(RELU ? pack_bf16x2(fmaxf(v0, 0.f), fmaxf(v1, 0.f)) : pack_bf16x2(v0, v1),
                                              yr, voff, so[mt] + (PCMS_STEM_VOFF ? 0 : rw * 128), 2);
        s1[0] += e0; s2[0] = fmaf(e0, e0, s2[0]);
        s1[1] += e1; s2[1] = fmaf(e1, e1, s2[1]);
      }
    }
  };

  // Every wave defers a box's epilogue to the next box: its 8 (wide) / 32 stores and BN sums are spread
  // over that box's 14 MFMA steps (3 items per step for steps 0-3, 2 after), so each SIMD's
  // store stream runs under the MFMAs instead of in bursts between them.
  f32x16_t prev[2][2];
  int pb = -1;  // box whose epilogue is still owed
  int b, bstep, bend;
  stem_box_walk(nbox, p.nbd, p.nbh * p.nbw, b, bstep, bend);
  // DENSE: box b's windows -> R buffer rb from halo buffer rb (two per thread)
  auto repack = [&](int rb) {
    const char* raw = lds + rb * kSDHaloBytes;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int j = tid + k * kSDThr;
      if (j < (bd + 2) * HH * 16) {
        const int row = j >> 4, w = j & 15;
        const u32x4_t* src = reinterpret_cast<const u32x4_t*>(raw + (row * HW + w) * 16);
        const u32x4_t a = src[0], bb = src[1], c = src[2];
        const u32x4_t r1 = {a[0], a[1], __builtin_amdgcn_perm(bb[0], a[2], 0x05040100u),
                            __builtin_amdgcn_perm(bb[1], bb[0], 0x05040302u)};
        const u32x4_t r2 = {__builtin_amdgcn_perm(bb[2], bb[1], 0x05040302u), c[0], c[1], c[2] & 0xffffu};
        char* dst = lds + kSD2R + rb * kSDRBytes + j * 32;
        const int sw = ((w >> 3) & 1) * 16;
        *reinterpret_cast<u32x4_t*>(dst + sw) = r1;
        *reinterpret_cast<u32x4_t*>(dst + (16 - sw)) = r2;
      }
    }
  };
  if (b < bend) stage(b, 0);
  if (DENSE && b + bstep < bend) stage(b + bstep, 1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if constexpr (DENSE) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (b < bend) repack(0);
  }
  for (int it = 0; b < bend; b += bstep, ++it) {
    // halo(b) has landed for this wave (vmcnt at the loop end); barrier: for all waves, and
    // every wave is done reading the buffer the next DMA overwrites.  A raw s_barrier, not
    // __syncthreads(): its fence would wait vmcnt(0), draining this wave's output stores
    // every box instead of leaving them in flight under the next box's MFMAs.  (The halo DMA
    // is inline asm, invisible to the compiler's wait insertion, for the same reason.)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    STEM_STAMP(0);
    const int bn = b + bstep;
    // DENSE: halo(b + 2G) into the buffer halo(b) left (repacked during the previous box);
    // halo(b + G) landed at the previous box's end and is repacked during this box's MFMAs
    if constexpr (DENSE) {
      if (bn + bstep < bend) stage(bn + bstep, it & 1);
    } else {
      if (bn < bend) stage(bn, (it + 1) & 1);
    }
    const int rp = DENSE && bn < bend ? (it + 1) & 1 : -1;  // R / halo buffer repacked this box
    const int rcur = (it & 1) * kSDRBytes;                  // DENSE: this box's R buffer
    STEM_STAMP(1);
    const bool interleave = pb >= 0 && is_full(pb);
    if (pb >= 0 && !interleave) epilogue(prev, pb);
    uint32_t pso[2] = {0u, 0u};
    if (interleave) tile_so(pb, pso);
    STEM_STAMP(2);
    const char* hl = lds + (it & 1) * kSDHaloBytes;
    f32x16_t acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[i][j][e] = bias_l[j];
    auto mfma_steps = [&](auto il) {
      constexpr bool IL = decltype(il)::value;
      int hs16 = hsel * 16;
      asm volatile("" : "+v"(hs16));
      auto load_a = [&](int st, s16x8_t (&a)[2]) {
        if constexpr (DENSE) {  // tap row (kd, kh) = (st / 3, st % 3): a whole-row offset in R
          const int off = ((st / 3) * HH + st % 3) * 16 * 32;
#pragma unroll
          for (int mt = 0; mt < 2; ++mt) a[mt] = *reinterpret_cast<const s16x8_t*>(lds + rcur + hb16[mt] + off);
          return;
        }
        const int o0 = tap_off(2 * st, HH, HW), o1 = tap_off(2 * st + 1, HH, HW);
        const int off16 = o0 * 16 + hs16 * (o1 - o0);
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) a[mt] = *reinterpret_cast<const s16x8_t*>(hl + hb16[mt] + off16);
      };
      auto load_b = [&](int st, s16x8_t (&w)[2]) {
        w[0] = *reinterpret_cast<const s16x8_t*>(wl + st * 64 * 32);
        w[1] = *reinterpret_cast<const s16x8_t*>(wl + (st * 64 + 32) * 32);
      };
      s16x8_t abuf[2][2], bbuf[2][2];
      load_a(0, abuf[0]);
      load_b(0, bbuf[0]);
#pragma unroll
      for (int st = 0; st < KS; ++st) {
        if (st + 1 < KS) {
          load_a(st + 1, abuf[(st + 1) & 1]);
          load_b(st + 1, bbuf[(st + 1) & 1]);
        }
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
#ifdef STEM_MFMA_STEPS  // ablation builds (tests/tools/ab_build.sh): MFMAs of the first N steps only
          if (st < STEM_MFMA_STEPS)
#endif
          {
            acc[mt][0] = mfma(abuf[st & 1][mt], bbuf[st & 1][0], acc[mt][0]);
            acc[mt][1] = mfma(abuf[st & 1][mt], bbuf[st & 1][1], acc[mt][1]);
          }
        }
        // the next step's four fragment reads go out ahead of this step's MFMAs (left to
        // itself the scheduler sank them below three of the MFMAs, exposing the LDS
        // latency); the owed epilogue items go between the MFMAs
        if (st + 1 < KS) __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
        if constexpr (IL) {
          // the 32 owed items over the KS steps (<= 4 per step: one per MFMA)
          constexpr int q14[15] = {0, 3, 6, 9, 12, 14, 16, 18, 20, 22, 24, 26, 28, 30, 32};
          constexpr int q9[10] = {0, 4, 8, 12, 16, 20, 24, 27, 30, 32};
          const int qa = DENSE ? q9[st] : q14[st], qb = DENSE ? q9[st + 1] : q14[st + 1];
#pragma unroll
          for (int q = qa; q < qb; ++q) item_full(prev, q >> 4, q & 15, pso);
#pragma unroll
          for (int q = qa; q < qb; ++q) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // 1 MFMA
            if constexpr (PCMS_STEM_WIDE) {
              if ((q & 3) == 3) {
                __builtin_amdgcn_sched_group_barrier(0x002, 7 + 16, 0);  // pack + BN sums + transpose
                __builtin_amdgcn_sched_group_barrier(0x040, 1, 0);       // 1 store (8 rows)
              } else {
                __builtin_amdgcn_sched_group_barrier(0x002, 7, 0);       // pack + BN sums
              }
            } else {
              __builtin_amdgcn_sched_group_barrier(0x002, 7, 0);  // pack + BN sums
              __builtin_amdgcn_sched_group_barrier(0x040, 1, 0);  // 1 store
            }
          }
          const int rest = 4 - (qb - qa);  // the step's other MFMAs (a constant once unrolled)
          if (rest == 1) __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          else if (rest == 2) __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
          else if (rest == 3) __builtin_amdgcn_sched_group_barrier(0x008, 3, 0);
        } else {
          __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
        }
        if (DENSE && st == 1 && rp >= 0) repack(rp);  // the next box's windows, under these MFMAs
        __builtin_amdgcn_sched_barrier(0);
      }
    };
    if (interleave) {
      mfma_steps(std::true_type{});
      cnt += 32.f;
    } else {
      mfma_steps(std::false_type{});
    }
    STEM_STAMP(3);
    if (it == 0) {  // BN shift: the first box's first voxel, per channel
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) K[nt] = __shfl(acc[0][nt][0], r_lane, 64);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) prev[i][j] = acc[i][j];
    pb = b;
    STEM_STAMP(4);
    // the next halo's DMA was issued before the 32 stores of the owed epilogue (none in the
    // first iteration)
    if (it == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if (PCMS_STEM_WIDE) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
    STEM_STAMP(5);
  }
  if (pb >= 0) epilogue(prev, pb);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  STEM_STAMP_END();
  if (!p.stats) return;
  // per wave (lanes r_lane and r_lane + 32 share channels and K): S = sum d + n K,
  // M2 = sum d^2 - (sum d)^2 / n; then Chan across the 8 waves
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
    float* cnts = p.stats + (long)mrows * 128;  // row counts after the [mrows][64][2] block
    if (tid == 0) cnts[blockIdx.x] = Nn;
    // zero this workgroup's share of the rows past gridDim.x
    for (int r = blockIdx.x + gridDim.x; r < mrows; r += gridDim.x) {
      p.stats[((long)r * 64 + tid) * 2] = 0.f;
      p.stats[((long)r * 64 + tid) * 2 + 1] = 0.f;
      if (tid == 0) cnts[r] = 0.f;
    }
  }
}


// Streaming stem weight gradient (the HBM-bound hot case: D % 4 == H % 4 == W % 16 == 0).
// dW[co][c][t] = sum_v dy[v][co] x[v + t][c]: GEMM with M = 64 co, N = 224 (tap, channel)
// columns, K = voxels.  Persistent: one 8-wave workgroup per CU walks 4x4x16 voxel boxes
// b = blockIdx.x + k gridDim.x.  Each box's dy tile (256 voxels x 128 B) and x halo
// (6x6x18 rows x 16 B) arrive by buffer LDS-DMA (inline asm, see dma16) into a 3-slot ring:
// two boxes in flight while one computes, counted vmcnt + raw s_barrier, every source
// offset a per-thread constant + the box base; the 43 DMA instructions of a box are spread
// over the 8 waves (5-6 each).  Wave w = (ks, ct) owns co tile ct = w & 1 and k-steps ks,
// ks + 4, ks + 8, ks + 12 (ks = w >> 1) of every box, with its 7 column tiles (112
// accumulators): two waves per SIMD, so one wave's MFMAs run while the other waits on its
// DMA issue or its LDS reads (ds_read_b64_tr_b16 transposes both operands; a B fragment is
// read by the two co-tile waves of its k-step).
// Flush: one fp32 partial row [64][cin_w][27] per workgroup (plain stores), summed into dw
// by stem_wgrad_reduce_kernel (deterministic, no atomics).
constexpr int kSWT = 512;                                  // 8 waves, two per SIMD
constexpr int kSWW = kSWT / 64;
// BD = box depth (boxes BD x 4 x 16), NS = ring slots (NS - 1 boxes in flight)
template <int BD, int NT = kSWT> struct SWGeom {
  static constexpr int BV = BD * 64;                            // voxels per box
  static constexpr int HV = (BD + 2) * 6 * 18;                  // halo rows (16 B)
  static constexpr int HRows = (HV + 63) / 64 * 64;             // rows written
  static constexpr int Buf = BV * 128 + HRows * 16;             // bytes per ring slot
  static constexpr int DYP = BV * 8 / NT;                       // dy DMA pieces per thread
  static constexpr int XI = (HRows / 64 + NT / 64 - 1) / (NT / 64);  // halo DMA rounds per wave (max)
};
constexpr int kSWBD = 4;  // box depth (2-deep boxes in 6 slots measured slower)
constexpr int kSWNS = 3;
constexpr int kSWLaneStride = 20;                        // flush: floats per lane (16 used)
constexpr int kSWRegion = 14 * 64 * kSWLaneStride * 4;   // 14 tiles (2 co x 7 columns), lane-major
constexpr int kSWRing = kSWNS * SWGeom<kSWBD>::Buf;
constexpr int kSWLds = kSWRing > 2 * kSWRegion ? kSWRing : 2 * kSWRegion;
static_assert(kSWLds <= 160 * 1024, "ring / flush regions fit in LDS");
// DENSE (<= 5 input channels): the MFMA columns are (tap row (kd, kh), k = 5 kw + c) -- 9 x 16
// = 144 in 5 column tiles instead of (tap, channel) = 28 x 8 in 7 -- over the R1 | R2 windows
// of the x halo (the forward's layout: one 32-B row per (halo d, halo h, w), halves swapped on
// w bit 3), repacked after each box's halo lands (one more barrier per box).  R after the ring.
constexpr int kSWRRows = (kSWBD + 2) * 6 * 16;
constexpr int kSWR = kSWRing;
constexpr int kSWLdsD = (kSWRing + kSWRRows * 32) > 2 * kSWRegion ? kSWRing + kSWRRows * 32 : 2 * kSWRegion;
static_assert(kSWLdsD <= 160 * 1024, "ring + windows / flush regions fit in LDS");

// BN: the stem's BatchNorm + ReLU backward apply fused in (models/unet3d.py:29-33: inc's
// conv.0 -> bn -> relu).  ``dy`` is then the gradient of the ReLU output (da) and ``bn.y``
// the stem's pre-BN output: the ring receives the da tile by LDS-DMA as before, each thread
// loads the y chunks it transforms into registers one box ahead (issued between the two
// boxes' DMA, so the counted vmcnt waits are unchanged), and after the box's DMA has landed
// the tile is rewritten in place as dy = k1 g + k2 xhat + k3, g = da [y sc + sh > 0]
// (bn_relu_bwd_apply_kernel's arithmetic): the stem's dy is never stored in HBM (its only
// consumer is this kernel: the input needs no gradient).
struct StemBN {
  const bf16_t* y;
  const float *scale, *shift, *mean, *invstd, *coef;
};
template <int BD, int NS, bool BN, bool DENSE = false>
__global__ void __launch_bounds__(kSWT, 1) stem_wgrad_stream_kernel(const bf16_t* x, const bf16_t* dy, float* part,
                                                                    int N, int D, int H, int W, int cin_w,
                                                                    uint32_t xbytes, uint32_t dybytes, StemBN bn) {
  constexpr int NT = DENSE ? 5 : 7;  // MFMA column tiles
  typedef SWGeom<BD> Gm;
  constexpr int BH = 4, BW = 16, HH = BH + 2, HW = BW + 2;
  constexpr int kSWBV = Gm::BV, kSWHV = Gm::HV, kSWBuf = Gm::Buf;
  constexpr int XI = Gm::XI;
  extern __shared__ __attribute__((aligned(16))) char swl[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ct = wave & 1, ks = wave >> 1;
  const int hsel = lane >> 5;
  const int nbw = W / BW, nbh = H / BH, nbd = D / BD;
  const int nbox = N * nbd * nbh * nbw;
  const i32x4_t xr = buffer_desc(x, xbytes);
  const i32x4_t dr = buffer_desc(dy, dybytes);

  // per-thread DMA source offsets relative to the box origin (constant over boxes)
  uint32_t dyrel[Gm::DYP];
#pragma unroll
  for (int i = 0; i < Gm::DYP; ++i) {
    const int pc = tid + i * kSWT;
    const int r = pc >> 3, q = pc & 7;
    const int ql = q ^ (((r >> 1) & 1) << 2);  // dy_off_bf16: 64-B halves swapped on odd row pairs
    const int rd = r >> 6, rh = (r >> 4) & 3, rw = r & 15;
    dyrel[i] = (uint32_t)(((rd * H + rh) * W + rw) * 128 + ql * 16);
  }
  // halo pieces of this wave: rows wave*64 + lane + kSWT i < HRows (XI or XI - 1 of them)
  const int nxp = (Gm::HRows / 64 - wave + kSWW - 1) / kSWW;
  int xrel[XI], xco[XI];
#pragma unroll
  for (int i = 0; i < XI; ++i) {
    const int hv = wave * 64 + lane + i * kSWT;
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
    for (int i = 0; i < Gm::DYP; ++i) dma16_nt(dr, lb + i * kSWT * 16, dyrel[i], so);
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
      dma16(xr, lb + kSWBV * 128 + i * kSWT * 16, voff, 0);
    }
  };

  // BN transform: every wave rewrites exactly the dy elements its own MFMAs read -- wave
  // (ks, ct) reads channels [32 ct, 32 ct + 32) of the rows of k-steps ks + 4 i, i < BD (rows
  // 16 (ks + 4 i) + rs, rs < 16), so no other wave waits for it (no workgroup barrier between
  // the transform and the MFMAs).  Lane: 16-B chunk q = lane & 3 of the row's 64-B half
  // (channels 32 ct + 8 q ..), rs = lane >> 2; dy_off_bf16's half swap depends on row bit 1 =
  // rs bit 1 only, so the lane's LDS column and its 8 channels' coefficients are fixed.
  constexpr int kTR = BD;
  const int tq = lane & 3, trs = lane >> 2;
  const int tcol = ((ct ^ ((trs >> 1) & 1)) * 64) + tq * 16;  // byte offset in the 128-B row
  const int tch = ct * 32 + tq * 8;                            // first logical channel
  float bsc[8], bsh[8], bmu[8], bk1[8], bka[8], bk3[8];  // bka = k2 invstd
  u32x4_t yreg[kTR];
  if constexpr (BN) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = tch + j;
      bsc[j] = bn.scale[c]; bsh[j] = bn.shift[c]; bmu[j] = bn.mean[c];
      bk1[j] = bn.coef[3 * c]; bka[j] = bn.coef[3 * c + 1] * bn.invstd[c]; bk3[j] = bn.coef[3 * c + 2];
    }
  }
  // y chunks of box b into registers (plain global loads: counted by vmcnt like the DMA);
  // row 16 (ks + 4 i) + rs of the box = voxel (d0 + i, h0 + ks, w0 + rs)
  auto load_y = [&](int b) {
    int n, d0, h0, w0;
    origin(b, n, d0, h0, w0);
    const long vb = ((long)(n * D + d0) * H + h0 + ks) * W + w0 + trs;
#pragma unroll
    for (int k = 0; k < kTR; ++k) {
      const bf16_t* src = bn.y + (vb + (long)k * H * W) * 64 + tch;
      yreg[k] = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(src));
    }
  };
  auto transform = [&](char* buf) {
#pragma unroll
    for (int k = 0; k < kTR; ++k) {
      u32x4_t* cp = reinterpret_cast<u32x4_t*>(buf + (16 * (ks + 4 * k) + trs) * 128 + tcol);
      const u32x4_t gv = *cp;
      float ga[8], yv[8], o[8];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        ga[2 * i] = __uint_as_float(gv[i] << 16); ga[2 * i + 1] = __uint_as_float(gv[i] & 0xffff0000u);
        yv[2 * i] = __uint_as_float(yreg[k][i] << 16); yv[2 * i + 1] = __uint_as_float(yreg[k][i] & 0xffff0000u);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float gg = (yv[j] * bsc[j] + bsh[j] > 0.f) ? ga[j] : 0.f;
        o[j] = bk1[j] * gg + (bka[j] * (yv[j] - bmu[j]) + bk3[j]);  // centred: no cancellation at |mean| >> std
      }
      u32x4_t ov;
#pragma unroll
      for (int i = 0; i < 4; ++i) ov[i] = pack_bf16x2(o[2 * i], o[2 * i + 1]);
      *cp = ov;
    }
  };

  const int g = (lane >> 4) & 1, qq = (lane & 15) >> 2, pp = lane & 3;
  f32x16_t acc[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[j][e] = 0.f;
  // lane offsets of the tr reads, with the wave's k-step offset folded in (k-step s = ks +
  // 4 i is box row (rd = i, rh = ks): dy rows at s * 2048, halo rows at (i HH + ks) HW)
  const int aoff = dy_off_bf16(8 * hsel + qq, ct * 32 + g * 16 + pp * 4) + ks * 2048;
  int boff[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    if constexpr (DENSE) {
      // column tile j: tap row tr = 2 j + g (tile 4's upper half re-reads row 8: dropped in the
      // flush), k = 4 pp .. + 3 = 8 B of the 32-B window row (hd = i + kd, hh = ks + kh, w =
      // 8 hsel + qq: the halves swapped on w bit 3 = hsel); relative to the window region
      const int trow = min(2 * j + g, 8), kd = trow / 3, kh = trow % 3;
      boff[j] = ((kd * HH + kh + ks) * 16 + 8 * hsel + qq) * 32 + (((pp >> 1) ^ hsel) * 16) + (pp & 1) * 8;
    } else {  // column tile j: taps 4 j + 2 g + (pp >> 1), channels 4 (pp & 1) .. + 3
      boff[j] = kSWBV * 128 + (8 * hsel + qq + tap_off(4 * j + 2 * g + (pp >> 1), HH, HW) + ks * HW) * 16 + (pp & 1) * 8;
    }
  }
#ifndef STEM_WG_TILES  // ablation builds: MFMAs of the first N column tiles only
#define STEM_WG_TILES 99
#endif
  constexpr int NTM = STEM_WG_TILES < NT ? STEM_WG_TILES : NT;
  auto compute = [&](const char* buf) {
    const uint32_t bbase = DENSE ? lds_addr(swl) + kSWR : lds_addr(buf);
    uint32_t pa = lds_addr(buf) + aoff, pb[7];
#pragma unroll
    for (int j = 0; j < NT; ++j) pb[j] = bbase + boff[j];
    if constexpr (DENSE)
      asm volatile("" : "+v"(pa), "+v"(pb[0]), "+v"(pb[1]), "+v"(pb[2]), "+v"(pb[3]), "+v"(pb[4]));
    else
      asm volatile("" : "+v"(pa), "+v"(pb[0]), "+v"(pb[1]), "+v"(pb[2]), "+v"(pb[3]), "+v"(pb[4]), "+v"(pb[5]),
                   "+v"(pb[6]));
    auto tr = [](uint32_t p, int off) {
      return __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4_t*)(uintptr_t)(p + off));
    };
    auto cat = [](s16x4_t lo, s16x4_t hi) { return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7); };
    auto load = [&](int i, s16x8_t& a, s16x8_t (&bq)[NT]) {
      const int dyb = i * 4 * 2048;
      // box d-row i: halo rows i HH HW (16 B) / window rows i HH 16 (32 B); the lane's second
      // voxel 4 w further
      const int hrb = DENSE ? i * HH * 16 * 32 : i * HH * HW * 16;
      constexpr int w4 = DENSE ? 4 * 32 : 4 * 16;
      a = cat(tr(pa, dyb), tr(pa, dyb + 512));
#pragma unroll
      for (int j = 0; j < NT; ++j) bq[j] = cat(tr(pb[j], hrb), tr(pb[j], hrb + w4));
    };
    s16x8_t a[2], bq[2][NT];
    load(0, a[0], bq[0]);
#pragma unroll
    for (int i = 0; i < BD; ++i) {
      if (i + 1 < BD) load(i + 1, a[(i + 1) & 1], bq[(i + 1) & 1]);
#pragma unroll
      for (int j = 0; j < NTM; ++j) acc[j] = mfma(a[i & 1], bq[i & 1][j], acc[j]);
    }
  };
  // DENSE: box halo (ring slot buf) -> the R1 | R2 windows (two per thread)
  auto repack = [&](const char* buf) {
    const char* raw = buf + kSWBV * 128;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int j = tid + k * kSWT;
      if (j < (BD + 2) * HH * 16) {
        const int row = j >> 4, w = j & 15;
        const u32x4_t* src = reinterpret_cast<const u32x4_t*>(raw + (row * HW + w) * 16);
        const u32x4_t a = src[0], bb = src[1], c = src[2];
        const u32x4_t r1 = {a[0], a[1], __builtin_amdgcn_perm(bb[0], a[2], 0x05040100u),
                            __builtin_amdgcn_perm(bb[1], bb[0], 0x05040302u)};
        const u32x4_t r2 = {__builtin_amdgcn_perm(bb[2], bb[1], 0x05040302u), c[0], c[1], c[2] & 0xffffu};
        char* dst = swl + kSWR + j * 32;
        const int sw = ((w >> 3) & 1) * 16;
        *reinterpret_cast<u32x4_t*>(dst + sw) = r1;
        *reinterpret_cast<u32x4_t*>(dst + (16 - sw)) = r2;
      }
    }
  };

  int b, G, bend;  // G: this workgroup's box stride
  stem_box_walk(nbox, nbd, nbh * nbw, b, G, bend);
  static_assert(!BN || NS == 3, "the y loads sit between the DMA of two consecutive boxes");
#pragma unroll
  for (int k = 0; k < NS - 1; ++k) {
    if (b + k * G < bend) stage(b + k * G, k);
    if (BN && k == 0 && b < bend) load_y(b);  // order: DMA(b), y(b), DMA(b + G)
  }
  for (int it = 0; b < bend; b += G, ++it) {
    // retire box b's DMA (the NS - 2 boxes after it may stay in flight), then barrier:
    // every wave's share of box b has landed and every wave is done reading the slot
    // refilled below
    if (b + (NS - 2) * G < bend) {
      if (nxp == XI) asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NS - 2) * (Gm::DYP + XI)) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NS - 2) * (Gm::DYP + XI - 1)) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    const int b2 = b + (NS - 1) * G;
    if constexpr (DENSE) repack(swl + (it % NS) * kSWBuf);  // R is free: every wave passed the barrier
    if constexpr (BN) {
      // box b's da tile and y chunks have landed: this wave's dy in place, then the next box's
      // y loads (before the DMA of box b + 2 G: the wait above stays a count of that DMA alone)
      transform(swl + (it % NS) * kSWBuf);
      if (b + G < bend) load_y(b + G);
    }
    if (b2 < bend) stage(b2, (it + NS - 1) % NS);
    if constexpr (DENSE) {  // every thread's windows (and own dy) written before any MFMA reads them
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    } else if constexpr (BN) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // own dy writes before own reads
    }
    compute(swl + (it % NS) * kSWBuf);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // flush, two stages: the waves of k-step sets 0 / 1 store their 7 tiles lane-major into
  // regions 0 / 1 (tiles ct * 7 + j; 16 of every 20 floats per lane: conflict-free
  // ds_write_b128), the waves of sets 2 / 3 add theirs into the same regions, then every
  // thread writes region 0 + region 1 into the partial row (a fixed summation order:
  // (ks0 + ks2) + (ks1 + ks3))
  float* reg = reinterpret_cast<float*>(swl) + (ks & 1) * (kSWRegion / 4);
  if (ks < 2) {
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      float* dst = reg + ((ct * NT + j) * 64 + lane) * kSWLaneStride;
#pragma unroll
      for (int q = 0; q < 4; ++q)
        *reinterpret_cast<f32x4_t*>(dst + 4 * q) =
            (f32x4_t){acc[j][4 * q], acc[j][4 * q + 1], acc[j][4 * q + 2], acc[j][4 * q + 3]};
    }
  }
  __syncthreads();
  if (ks >= 2) {
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      float* dst = reg + ((ct * NT + j) * 64 + lane) * kSWLaneStride;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        f32x4_t v = *reinterpret_cast<f32x4_t*>(dst + 4 * q);
        v += (f32x4_t){acc[j][4 * q], acc[j][4 * q + 1], acc[j][4 * q + 2], acc[j][4 * q + 3]};
        *reinterpret_cast<f32x4_t*>(dst + 4 * q) = v;
      }
    }
  }
  __syncthreads();
  // partial row [64 co][cin_w][27]: element (co, column 8 t + c) sits in tile (co >> 5, col >> 5),
  // lane (col & 31) + 32 hs, register e, where (e & 3) + 8 (e >> 2) + 4 hs = co & 31
  const float* r0 = reinterpret_cast<const float*>(swl);
  const float* r1 = r0 + kSWRegion / 4;
  const int per_co = cin_w * 27;  // <= 216: thread (half h, rem) owns column rem of co rows [32 h, 32 h + 32)
  float* prow = part + (long)blockIdx.x * 64 * per_co;
  const int hh = tid >> 8, rem = tid & 255;
  if (rem < per_co) {
    const int c = rem / 27, t = rem - c * 27;
    // column of (tap t, channel c): 8 t + c; DENSE: 16 (tap row) + 5 kw + c
    const int col = DENSE ? 16 * (t / 3) + 5 * (t % 3) + c : 8 * t + c;
    const int cb = ((hh * NT + (col >> 5)) * 64 + (col & 31)) * kSWLaneStride;
#pragma unroll
    for (int cr = 0; cr < 32; ++cr) {
      const int hs = (cr >> 2) & 1, e = (cr & 3) + 4 * (cr >> 3);
      const int o = cb + 32 * hs * kSWLaneStride + e;
      prow[(hh * 32 + cr) * per_co + rem] = r0[o] + r1[o];
    }
  }
}

// dw[o] += sum over the workgroup partial rows (fixed order).  Block = 32 outputs x 8 row
// groups: 32 independent 128-B row segments in flight per thread group, LDS combine.
__global__ void __launch_bounds__(256) stem_wgrad_reduce_kernel(const float* part, int rows, int total, float* dw) {
  __shared__ float red[8][32];
  const int ol = threadIdx.x & 31, rg = threadIdx.x >> 5;
  const int o = blockIdx.x * 32 + ol;
  float s = 0.f;
  if (o < total) {
    // rows rg, rg + 8, ... summed in that order; loads issued 32 at a time ahead of the adds
    int r = rg;
    for (; r + 8 * 31 < rows; r += 8 * 32) {
      float v[32];
#pragma unroll
      for (int k = 0; k < 32; ++k) v[k] = part[(long)(r + 8 * k) * total + o];
#pragma unroll
      for (int k = 0; k < 32; ++k) s += v[k];
    }
    for (; r < rows; r += 8) s += part[(long)r * total + o];
  }
  red[rg][ol] = s;
  __syncthreads();
  if (rg == 0 && o < total) {
    float t = 0.f;
#pragma unroll
    for (int g2 = 0; g2 < 8; ++g2) t += red[g2][ol];
    dw[o] += t;
  }
}

}  // namespace

// the stem weight gradient's MFMA columns: 28 taps x 8 channels (0, the product: 125.2 vs
// 127.1 us for the dense form on one box) or dense tap rows x 16 for <= 5
// input channels (1: A/B); pcms_stem_wgrad_dense sets it
static int g_stem_wgrad_dense = 0;

// the dedicated stem kernels' shape conditions (other shapes take the general conv kernels)
static bool stem_fwd_direct_shape(int N, int D, int H, int W) {
  const Box b = fwd_box(D, H, W);
  return b.lbw == 4 && b.lbd + b.lbh == 5 && (b.lbd == 2 || b.lbd == 3) && (long)N * D * H * W * 128 < (long)kOOB;
}
static bool stem_wgrad_streams(int N, int D, int H, int W) {
  return D % kSWBD == 0 && H % 4 == 0 && W % 16 == 0 && (long)N * D * H * W * 128 < (1L << 31);
}

extern "C" {

int pcms_stem_pack(const float* w, void* out, int cin_w, hipStream_t s) {
  if (cin_w > 8) return -1;
  hipLaunchKernelGGL(stem_pack_kernel, dim3(cdiv(kStemPackElems, 256)), dim3(256), 0, s, w, (bf16_t*)out, cin_w);
  PCMS_CHECK_LAUNCH();
}
int pcms_stem_pack_elems(void) { return kStemPackElems; }

// the stem weight gradient's column form: 1 dense (tap row x 16, <= 5 channels), 0 tap x 8
// channels; v < 0 only queries.  Returns the previous setting (test / A/B switch)
int pcms_stem_wgrad_dense(int v) {
  const int old = g_stem_wgrad_dense;
  if (v >= 0) g_stem_wgrad_dense = v;
  return old;
}

// bit 0: pcms_stem_fwd runs this shape; bit 1: pcms_stem_wgrad runs it
int pcms_stem_supported(int N, int D, int H, int W) {
  return (stem_fwd_direct_shape(N, D, H, W) ? 1 : 0) | (stem_wgrad_streams(N, D, H, W) ? 2 : 0);
}

// BatchNorm statistics rows pcms_stem_fwd writes
int pcms_stem_fwd_rows(int N, int D, int H, int W) {
  // one row per workgroup of the persistent grid (round 6: was one per box, the rows past the
  // grid zero-filled by the kernel -- 2 MB of zeros and a two-launch finalize over 4096 rows at
  // config 2 instead of one launch over 256)
  const Box b = fwd_box(D, H, W);
  return std::min(N * cdiv(D, 1 << b.lbd) * cdiv(H, 1 << b.lbh) * cdiv(W, 1 << b.lbw), device_cus());
}

// x: (N, D, H, W, 8) bf16; y: (N, D, H, W, 64) bf16; stats rows = pcms_stem_fwd_rows
int pcms_stem_fwd(const void* x, const void* wpack, const float* bias, void* y, float* stats,
                  int N, int D, int H, int W, int flags, hipStream_t s) {
  if (!stem_fwd_direct_shape(N, D, H, W)) return -5;
  if (flags & ~(PCMS_CONV_RELU | PCMS_STEM_DENSE) || (stats && (flags & PCMS_CONV_RELU))) return -8;
  const bool relu = flags & PCMS_CONV_RELU, dense = flags & PCMS_STEM_DENSE;
  const Box b = fwd_box(D, H, W);
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
  const long xbytes = p.nvox * 16, ybytes = p.nvox * 128;
  const int grid = std::min(nbox, device_cus());
  auto kern = dense ? (b.lbd == 2 ? (relu ? stem_fwd_direct_kernel<2, 3, true, true> : stem_fwd_direct_kernel<2, 3, false, true>)
                                  : (relu ? stem_fwd_direct_kernel<3, 2, true, true> : stem_fwd_direct_kernel<3, 2, false, true>))
                    : (b.lbd == 2 ? (relu ? stem_fwd_direct_kernel<2, 3, true> : stem_fwd_direct_kernel<2, 3, false>)
                                  : (relu ? stem_fwd_direct_kernel<3, 2, true> : stem_fwd_direct_kernel<3, 2, false>));
  const int lds = dense ? kSD2Lds : kSDLds;
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  hipLaunchKernelGGL(kern, dim3(grid), dim3(kSDThr), lds, s, p, nbox, pcms_stem_fwd_rows(N, D, H, W), (uint32_t)xbytes,
                     (uint32_t)ybytes);
  PCMS_CHECK_LAUNCH();
}

// fp32 workspace floats pcms_stem_wgrad needs (0: shape not supported)
int pcms_stem_wgrad_ws_floats(int N, int D, int H, int W, int cin_w) {
  if (!stem_wgrad_streams(N, D, H, W)) return 0;
  const int nbox = N * (D / kSWBD) * (H / 4) * (W / 16);
  return std::min(nbox, device_cus()) * 64 * cin_w * 27;
}

// dw [64][cin_w][27] fp32 += stem weight gradient (x: 8-channel bf16 input, dy: 64 ch);
// ws: pcms_stem_wgrad_ws_floats(...) floats (one partial row per workgroup, fixed-order sum)
static int stem_wgrad_any(const void* x, const void* dy, float* dw, float* ws, int cin_w, int N, int D, int H,
                          int W, const StemBN& bn, hipStream_t s) {
  if (cin_w > 8 || cin_w < 1) return -1;
  if (!stem_wgrad_streams(N, D, H, W)) return -5;
  if (ws == nullptr) return -2;
  const int nbox = N * (D / kSWBD) * (H / 4) * (W / 16);
  const int grid = std::min(nbox, device_cus());
  const long xbytes = (long)N * D * H * W * 16, dybytes = (long)N * D * H * W * 128;
  const bool dense = cin_w <= 5 && g_stem_wgrad_dense;
  auto kern = bn.y ? (dense ? stem_wgrad_stream_kernel<kSWBD, kSWNS, true, true> : stem_wgrad_stream_kernel<kSWBD, kSWNS, true>)
                   : (dense ? stem_wgrad_stream_kernel<kSWBD, kSWNS, false, true> : stem_wgrad_stream_kernel<kSWBD, kSWNS, false>);
  const int lds = dense ? kSWLdsD : kSWLds;
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  hipLaunchKernelGGL(kern, dim3(grid), dim3(kSWT), lds, s, (const bf16_t*)x, (const bf16_t*)dy, ws, N, D, H, W,
                     cin_w, (uint32_t)xbytes, (uint32_t)dybytes, bn);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  const int total = 64 * cin_w * 27;
  hipLaunchKernelGGL(stem_wgrad_reduce_kernel, dim3(cdiv(total, 32)), dim3(256), 0, s, (const float*)ws, grid, total,
                     dw);
  PCMS_CHECK_LAUNCH();
}

int pcms_stem_wgrad(const void* x, const void* dy, float* dw, float* ws, int cin_w, int N, int D, int H, int W,
                    hipStream_t s) {
  return stem_wgrad_any(x, dy, dw, ws, cin_w, N, D, H, W, StemBN{}, s);
}

// the same with the stem's BatchNorm + ReLU backward apply fused in: da = the gradient of the
// stem block's first ReLU output, y = the stem's pre-BN output, BN forward coefficients and
// coef = pcms_bn_relu_bwd's apply coefficients (k1, k2, k3 per channel)
int pcms_stem_wgrad_bn(const void* x, const void* da, const void* y, const float* scale, const float* shift,
                       const float* mean, const float* invstd, const float* coef, float* dw, float* ws, int cin_w,
                       int N, int D, int H, int W, hipStream_t s) {
  if (!y || !scale || !shift || !mean || !invstd || !coef) return -2;
  return stem_wgrad_any(x, da, dw, ws, cin_w, N, D, H, W,
                        StemBN{(const bf16_t*)y, scale, shift, mean, invstd, coef}, s);
}

}  // extern "C"
