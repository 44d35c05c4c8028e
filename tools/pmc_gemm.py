#!/usr/bin/env python
"""Short GEMM driver for PMC collection (rocprofv3 --pmc ... -- python3 tools/pmc_gemm.py): the BERT-base FFN1
projection's forward (NT), data-gradient (NN) and weight-gradient (TN, f32) GEMMs on the 256-row pipelined kernel,
10 launches each. `python tools/pmc_gemm.py --summary <counter_collection.csv>...` prints the per-dispatch means per
kernel and the derived ratios (MFMA busy share, LDS bank-conflict share, wave-state split)."""
import collections
import csv
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run():
    import torch
    from distributed_tensorflow_amd.ops._util import call, ptr, stream, workspace
    dev = torch.device("cuda")
    M, N, K = 16384, 3072, 768
    x = torch.randn(M, K, device=dev).to(torch.bfloat16)
    w = torch.randn(N, K, device=dev).to(torch.bfloat16)
    dy = torch.randn(M, N, device=dev).to(torch.bfloat16)
    y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    dx = torch.empty(M, K, device=dev, dtype=torch.bfloat16)
    dw = torch.empty(N, K, device=dev, dtype=torch.float32)
    ws = workspace(dev)
    for _ in range(10):  # y = x w^T (NT)
        call("dtf_gemm256", ptr(x), ptr(w), ptr(y), M, N, K, K, K, N, 0, 0, 0, 1, ptr(ws), ws.numel(), stream())
    for _ in range(10):  # dx = dy w (NN: B = w stored [N][K] = [k][cols])
        call("dtf_gemm256", ptr(dy), ptr(w), ptr(dx), M, K, N, N, K, K, 0, 1, 0, 1, ptr(ws), ws.numel(), stream())
    for _ in range(10):  # dw = dy^T x (TN, f32; A = dy [M][N] = [k][rows], B = x [M][K] = [k][cols])
        call("dtf_gemm256", ptr(dy), ptr(x), ptr(dw), N, K, M, N, K, K, 1, 1, 1, 1, ptr(ws), ws.numel(), stream())
    torch.cuda.synchronize()


def summary(paths):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in paths:
        for r in csv.DictReader(open(p)):
            k = r.get("Kernel_Name", "?")[:70]
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in vals.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        print(k)
        for c in sorted(m):
            print(f"   {c:28s} {m[c]:16.0f}")
        if "SQ_WAVE_CYCLES" in m and m["SQ_WAVE_CYCLES"] > 0:
            wc = m["SQ_WAVE_CYCLES"]
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
                if c in m:
                    print(f"   {c + ' / WAVE_CYCLES':42s} {m[c] / wc:6.3f}")
        if "SQ_LDS_BANK_CONFLICT" in m and m.get("SQ_LDS_IDX_ACTIVE", 0) > 0:
            print(f"   LDS bank-conflict share of LDS cycles      {m['SQ_LDS_BANK_CONFLICT'] / m['SQ_LDS_IDX_ACTIVE']:6.3f}")
        if m.get("TCC_HIT_sum", 0) + m.get("TCC_MISS_sum", 0) > 0:
            print(f"   L2 hit rate                                {m['TCC_HIT_sum'] / (m['TCC_HIT_sum'] + m['TCC_MISS_sum']):6.3f}")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m and m.get("GRBM_GUI_ACTIVE", 0) > 0:
            # MFMA busy cycles summed over SIMDs vs (GPU-active cycles per XCD x 256 CUs x 4 SIMDs)
            per = m["GRBM_GUI_ACTIVE"] / 8
            print(f"   MFMA busy share (1024 SIMDs)               {m['SQ_VALU_MFMA_BUSY_CYCLES'] / (per * 1024):6.3f}")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--summary":
        summary(sys.argv[2:])
    else:
        run()
