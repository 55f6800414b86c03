"""Bit-for-bit comparison of the stem kernels of two builds of the library (test tooling):
the product library (or ``$2``) against a variant (``$1``; files under the package directory,
built by tests/tools/ab_build.sh).  A store / schedule change of pcms_stem_fwd or pcms_stem_wgrad_bn
must leave every output byte unchanged; prints one line per shape and exits non-zero on a
difference."""
import ctypes
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
FLAGS = int(os.environ.get("STEM_FLAGS", "16"))  # pcms_stem_fwd kernel choice (16: K-dense)
# outputs that must match (a box-walk change reorders the fp32 sums of stats / dw: "y,y_eval")
KEYS = os.environ.get("STEM_KEYS", "y,stats,y_eval,dw").split(",")
sys.path.insert(0, REPO)


def bind(path):
    from pcms_amd import _lib as L
    lib = ctypes.CDLL(path)

    def call(name, *args):
        sig = L.SIGNATURES[name]
        fn = getattr(lib, name)
        fn.argtypes = [L._CT[c] for c in sig]
        fn.restype = ctypes.c_int
        conv = [L.ptr(a) if c == "p" else a for c, a in zip(sig, args)]
        if sig.endswith("s"):
            conv.append(torch.cuda.current_stream().cuda_stream)
        rc = fn(*conv)
        if rc != 0 and sig.endswith("s"):
            raise RuntimeError(f"{name}: {rc}")
        return rc
    return call


def run(call, N, S, seed):
    g = torch.Generator().manual_seed(seed)
    nvox = N * S[0] * S[1] * S[2]
    T = torch.bfloat16
    x = torch.zeros(nvox, 8)
    x[:, :5] = torch.rand(nvox, 5, generator=g)
    x = x.to(T).cuda()
    w = (torch.randn(64, 5, 27, generator=g) * 0.2).cuda()
    bias = torch.randn(64, generator=g).cuda()
    wp = torch.empty(call("pcms_stem_pack_elems"), dtype=T, device="cuda")
    call("pcms_stem_pack", w, wp, 5)
    rows = call("pcms_stem_fwd_rows", N, *S)
    stats = torch.full((rows * 129,), float("nan"), device="cuda")
    y = torch.full((nvox * 64,), float("nan"), device="cuda").to(T)
    call("pcms_stem_fwd", x, wp, bias, y, stats, N, *S, FLAGS)
    ye = torch.full_like(y, float("nan"))
    call("pcms_stem_fwd", x, wp, bias, ye, None, N, *S, 2 | FLAGS)  # eval: folded BN + ReLU epilogue
    da = torch.randn(nvox * 64, generator=g).to(T).cuda()
    sc, sh = (torch.rand(64, generator=g) + 0.5).cuda(), (torch.randn(64, generator=g) * 0.1).cuda()
    mean, invstd = torch.randn(64, generator=g).cuda(), (torch.rand(64, generator=g) + 0.5).cuda()
    coef = torch.randn(192, generator=g).cuda()
    dw = torch.zeros(64 * 5 * 27, device="cuda")
    ws = torch.empty(call("pcms_stem_wgrad_ws_floats", N, *S, 5), device="cuda")
    call("pcms_stem_wgrad_bn", x, da, y, sc, sh, mean, invstd, coef, dw, ws, 5, N, *S)
    torch.cuda.synchronize()
    return {"y": y.view(torch.int16), "stats": stats, "y_eval": ye.view(torch.int16), "dw": dw}


def main():
    pkg = os.path.join(REPO, "prostate-cancer-multimodal-segmentation_amd")
    a = bind(os.path.join(pkg, sys.argv[2] if len(sys.argv) > 2 else "libpcms_hip.so"))
    b = bind(os.path.join(pkg, sys.argv[1]))
    bad = 0
    for N, S in ((1, (12, 16, 32)), (3, (4, 4, 16)), (1, (32, 64, 64)), (2, (128, 128, 64))):
        ra, rb = run(a, N, S, 7), run(b, N, S, 7)
        diff = {k: int((ra[k] != rb[k]).sum()) for k in ra if k != "stats"}
        diff["stats"] = int((ra["stats"].view(torch.int32) != rb["stats"].view(torch.int32)).sum())
        ok = all(diff[k] == 0 for k in KEYS)
        bad += not ok
        print(f"N={N} S={S}: {'bit-identical' if ok else 'DIFFERENT'} {diff}", flush=True)
        if diff["y"]:
            # where the forward outputs differ: histograms over the box-relative coordinates
            badm = (ra["y"] != rb["y"]).view(N, S[0], S[1], S[2], 64).cpu()
            idx = badm.nonzero()
            for name, col, mod in (("d%4", 1, 4), ("h%8", 2, 8), ("w%16", 3, 16), ("c//8", 4, None)):
                v = idx[:, col] % mod if mod else idx[:, col] // 8
                print(f"   {name}: {torch.bincount(v, minlength=mod or 8).tolist()}", flush=True)
            print(f"   d: {torch.bincount(idx[:, 1]).tolist()[:40]}", flush=True)
            print(f"   first: {idx[:8].tolist()}", flush=True)
            ya = ra["y"].view(N, S[0], S[1], S[2], 64)
            yb = rb["y"].view(N, S[0], S[1], S[2], 64)
            n, d, h, w, c = idx[0].tolist()
            print(f"   a[{n},{d},{h},{w}] = {ya[n, d, h, w].tolist()}", flush=True)
            print(f"   b[{n},{d},{h},{w}] = {yb[n, d, h, w].tolist()}", flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
