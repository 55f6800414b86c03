// Stem forward timeline (test tooling, not product): the product kernel built with its
// STEM_STAMP hooks writing s_memtime stamps per wave and box into spare LDS, copied out at
// the end.  Driven by tests/kexp/stem_tl.py.
#include <stdint.h>
#define STEM_TL_BOXES 16
#define STEM_STAMP(k)                                                                              \
  do {                                                                                             \
    const uint64_t t_ = __builtin_amdgcn_s_memtime();                                             \
    if (lane == 0 && it < STEM_TL_BOXES)                                                           \
      reinterpret_cast<uint64_t*>(lds + kSDLds)[(wave * STEM_TL_BOXES + it) * 8 + (k)] = t_;     \
  } while (0)
#define STEM_STAMP_END()                                                                           \
  do {                                                                                             \
    if (lane == 0) {                                                                               \
      const uint64_t* src_ = reinterpret_cast<const uint64_t*>(lds + kSDLds) + wave * STEM_TL_BOXES * 8; \
      uint64_t* dst_ = p.tl + ((long)blockIdx.x * 8 + wave) * STEM_TL_BOXES * 8;                   \
      for (int q_ = 0; q_ < STEM_TL_BOXES * 8; ++q_) dst_[q_] = src_[q_];                          \
    }                                                                                              \
  } while (0)
// the timeline pointer rides in a wrapper of the params struct
#include "../../prostate-cancer-multimodal-segmentation_amd/csrc/conv_common.h"
struct Conv3ParamsTL : Conv3Params { uint64_t* tl; };
#define Conv3Params Conv3ParamsTL
#define stem_fwd_direct_kernel stem_fwd_tl_kernel
#define pcms_stem_pack tl_stem_pack
#define pcms_stem_pack_elems tl_stem_pack_elems
#define pcms_stem_supported tl_stem_supported
#define pcms_stem_fwd_rows tl_stem_fwd_rows
#define pcms_stem_fwd tl_stem_fwd_unused
#define pcms_stem_wgrad_ws_floats tl_stem_wgrad_ws_floats
#define pcms_stem_wgrad tl_stem_wgrad
#include "../../prostate-cancer-multimodal-segmentation_amd/csrc/stem.hip"
#undef Conv3Params

extern "C" int exp_stem_fwd_tl(const void* x, const void* wpack, const float* bias, void* y, float* stats, uint64_t* tl,
                               int N, int D, int H, int W, hipStream_t s) {
  const Box b = fwd_box(D, H, W);
  Conv3ParamsTL p;
  p.x0 = x; p.x1 = nullptr; p.c0 = 8; p.c1 = 0;
  p.w = wpack; p.bias = bias; p.y0 = y; p.y1 = nullptr; p.cy0 = 64;
  p.yacc = nullptr; p.stats = stats; p.accumulate = 0;
  p.N = N; p.D = D; p.H = H; p.W = W; p.Cin = 8; p.Cout = 64;
  p.nvox = (long)N * D * H * W;
  p.nchunk = 1; p.chunks_per_split = 1;
  p.lbd = b.lbd; p.lbh = b.lbh; p.lbw = b.lbw;
  p.nbd = cdiv(D, 1 << b.lbd); p.nbh = cdiv(H, 1 << b.lbh); p.nbw = cdiv(W, 1 << b.lbw);
  p.tl = tl;
  const int nbox = N * p.nbd * p.nbh * p.nbw;
  const long xbytes = p.nvox * 16, ybytes = p.nvox * 128;
  const int grid = std::min(nbox, device_cus());
  auto kern = b.lbd == 2 ? stem_fwd_tl_kernel<2, 3> : stem_fwd_tl_kernel<3, 2>;
  const int lds = kSDLds + 8 * STEM_TL_BOXES * 8 * 8;
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  hipLaunchKernelGGL(kern, dim3(grid), dim3(kSDThr), lds, s, p, nbox, nbox, (uint32_t)xbytes, (uint32_t)ybytes);
  return (int)hipGetLastError();
}
