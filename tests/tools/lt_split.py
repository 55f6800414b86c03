"""layer_times with the engine's split-K threshold overridden (diagnostic):
    python tests/tools/lt_split.py THRESHOLD TARGET"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import pcms_amd  # noqa: E402
from pcms_amd import engine  # noqa: E402
from pcms_amd._lib import query  # noqa: E402

THR, TGT = int(sys.argv[1]), int(sys.argv[2])


def _splits(self, N, S, cin, cout, code):
    mb = query("pcms_conv3_mblocks", N, *S)
    wgs = mb * (cout // 64)
    nch = -(-cin // query("pcms_conv3_chunk", code))
    if wgs >= THR or nch == 1 or wgs == 0:
        return 1
    return max(1, min(nch, -(-TGT // wgs)))


engine.UNetEngine._splits = _splits
sys.argv = [sys.argv[0]]
import layer_times  # noqa: E402
layer_times.main()
