#!/usr/bin/env python
"""Short conv driver for PMC collection (rocprofv3 --pmc ... -- python3 tools/pmc_conv.py): ResNet-50 stage-1 3x3
forward (64 -> 64, the general 128x64 tap-uniform tile), stage-3 1x1 reducing forward (1024 -> 256) and the
stage-1 channel-expanding pointwise forward (pwconv.hip), 10 launches each, BN statistics on as in the model.
`python tools/pmc_conv.py --summary <counter_collection.csv>...` prints per-kernel means and the derived ratios
(tools/pmc_gemm.py)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run():
    import torch
    from distributed_tensorflow_amd.ops._util import IntOut, call, ptr, stream
    dev = torch.device("cuda")
    BF = torch.bfloat16
    rows = IntOut()
    for (N, H, C, K, R, pad) in ((256, 56, 64, 64, 3, 1), (256, 14, 1024, 256, 1, 0), (256, 56, 64, 256, 1, 0)):
        x = (torch.rand(N, H, H, C, device=dev) * 2 - 1).to(BF)
        w = ((torch.rand(K, R, R, C, device=dev) * 2 - 1) * 0.1).to(BF)
        P = H + 2 * pad - R + 1
        y = torch.empty(N, P, P, K, device=dev, dtype=BF)
        part = torch.empty(((N * P * P + 63) // 64) * 2 * K, device=dev)
        for _ in range(10):
            call("dtf_conv_fwd", ptr(x), ptr(w), ptr(y), None, ptr(part), rows.addr, N, H, H, C, K, R, R, P, P, 1, 1,
                 pad, pad, 1, 1, 0, 0, -1, stream())
        torch.cuda.synchronize()
        del x, w, y, part


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--summary":
        from pmc_gemm import summary  # noqa: E402
        summary(sys.argv[2:])
    else:
        run()
