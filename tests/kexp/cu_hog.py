"""What RCCL kernels beside the backward do to the persistent one-workgroup-per-CU kernels
(test tooling): K spinning workgroups (tests/kexp/cu_hog.hip, 24 KiB of LDS each, so no
persistent workgroup fits beside one) hold K CUs on a side stream for the whole of a bench
training step; the step is timed with HIP events on its own stream, with the persistent
grids at all CUs (reserve 0) and with pcms_set_cu_reserve(R).

    make -C tests/kexp libcuhog.so && python tests/kexp/cu_hog.py [K,K,...] [R,R,...]
"""
import ctypes
import os
import statistics
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))


def main():
    ks = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "0,1,4,8,32").split(",")]
    import pcms_amd  # noqa: F401
    from pcms_amd.synthetic import make_batch
    from pcms_amd.utils.trainer import Trainer
    hog = ctypes.CDLL(os.path.join(HERE, "libcuhog.so"))
    hog.cu_hog.argtypes = [ctypes.c_int, ctypes.c_double, ctypes.c_void_p, ctypes.c_void_p]
    torch.manual_seed(0)
    tr = Trainer({"device": "cuda", "learning_rate": 1e-4, "batch_size": 2, "num_epochs": 1,
                  "loss": "bce_dice", "precision": "bf16"})
    b = make_batch(2, (128, 128, 64), seed=1)
    batch = {"image": b["image"].cuda(), "label": b["label"].cuda()}
    sink = torch.zeros(64, dtype=torch.int32, device="cuda")
    side = torch.cuda.Stream()
    for _ in range(3):
        tr.step(batch)
    torch.cuda.synchronize()
    # per-launch cost with a kernel resident on another queue: 400 dependent tiny launches (a
    # 4-element fill) on the compute stream, with and without one hog workgroup beside them
    tiny = torch.zeros(4, device="cuda")
    for k in sorted(set([0, 1] + ks)):
        ts = []
        for _ in range(3):
            side.wait_stream(torch.cuda.current_stream())
            hog.cu_hog(k, 4000.0, sink.data_ptr(), side.cuda_stream)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(400):
                tiny.add_(1.0)
            e1.record()
            e1.synchronize()
            torch.cuda.current_stream().wait_stream(side)
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3 / 400)
        print(f"hog {k:3d} CUs:  {statistics.median(ts):6.2f} us per dependent tiny launch (all {[round(t, 2) for t in ts]})",
              flush=True)
    for k in ks:
        ts = []
        for _ in range(5):
            side.wait_stream(torch.cuda.current_stream())
            hog.cu_hog(k, 16000.0, sink.data_ptr(), side.cuda_stream)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            tr.step(batch)
            e1.record()
            e1.synchronize()
            torch.cuda.current_stream().wait_stream(side)
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        print(f"hog {k:3d} CUs:  step {statistics.median(ts):7.3f} ms  (all {[round(t, 2) for t in ts]})", flush=True)


if __name__ == "__main__":
    main()
