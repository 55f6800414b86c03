"""TEMP: per-workgroup s_memrealtime stamps of the bf16 weight gradient (100 MHz clock)."""
import ctypes, os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import pcms_amd
from pcms_amd import _lib as L
lib = L.load()
lib.pcms_conv3_wgrad_dbg.argtypes = [ctypes.c_void_p]
for (N, D, H, W, c0, co) in [(2, 8, 8, 4, 1024, 1024), (2, 8, 8, 4, 512, 1024), (2, 16, 16, 8, 512, 512), (2, 128, 128, 64, 64, 64)]:
    x0 = torch.randn(N * D * H * W * c0, device="cuda").to(torch.bfloat16)
    dy = torch.randn(N * D * H * W * co, device="cuda").to(torch.bfloat16)
    dw = torch.zeros(co * c0 * 27, device="cuda")
    ws = torch.empty(max(1, L.query("pcms_conv3_wgrad_ws_floats", 1, N, D, H, W, c0, 0, co, 256)), device="cuda")
    dbg = torch.zeros(8192 * 16, dtype=torch.int64, device="cuda")
    for it in range(3):
        lib.pcms_conv3_wgrad_dbg(dbg.data_ptr() if it == 2 else None)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        L.call("pcms_conv3_wgrad", 1, x0, c0, None, 0, dy, dw, ws, N, D, H, W, co, c0, 256, 1)
        e.record(); torch.cuda.synchronize()
    lib.pcms_conv3_wgrad_dbg(None)
    t = dbg.view(-1, 16).cpu()
    nwg = int((t[:, 0] > 0).sum())
    t = t[:nwg].double()
    t0 = t[:, 0].min()
    rel = (t - t0) / 100.0  # us
    print(f"{c0}->{co} {D}x{H}x{W}: {nwg} WGs, kernel {s.elapsed_time(e)*1e3:.1f} us", flush=True)
    import statistics
    def med(a): return statistics.median(a.tolist())
    st = rel[:, 0]
    print(f"  start spread {st.min():.1f}..{st.max():.1f} us; per-WG phases (median): "
          f"stage0 {med(rel[:,1]-rel[:,0]):.1f}, box0 {med(rel[:,2]-rel[:,1]):.1f}, wait0 {med(rel[:,3]-rel[:,2]):.1f}, "
          f"box1 {med(rel[:,4]-rel[:,3]):.1f}, wait1 {med(rel[:,5]-rel[:,4]):.1f}, to_flush {med(rel[:,10]-rel[:,1]):.1f}, "
          f"flush {med(rel[:,11]-rel[:,10]) if (rel[:,11]>0).any() else -1:.1f}, total {med(rel[:,11]-rel[:,0]) if (rel[:,11]>0).any() else med(rel[:,10]-rel[:,0]):.1f}", flush=True)
