#!/usr/bin/env python3
"""Per-kernel achieved TFLOP/s and TB/s of the 1-GPU Wide&Deep step against MI355X peaks, from a
rocprofv3 kernel trace (``--kernel-trace --output-format csv``) of bench.py:

    python tools/kernel_roofline.py gpurun_out/prof/run_kernel_trace.csv --U 212000 > profiles/...

Kernels are identified by name + grid size and given the FLOPs / bytes of their W&D call (batch
16384, 26 x 32-d embeddings + 13 dense, MLP 896(ext)-1024-512-256-1, bias-folded K of 1032 / 520,
weight-gradient split-K slabs); ``U`` = unique keys per batch (--measure-U). Durations
are medians over the steady steps (the first 3 steps are skipped). Bytes are the compulsory
traffic (each operand read once, outputs written once), so TB/s is a lower bound on what the
kernel moved. Peaks: 2.5 PFLOP/s dense bf16 MFMA, 8 TB/s HBM3E."""
import argparse
import csv
import re
import statistics

PEAK_TF, PEAK_TB = 2500.0, 8.0
B, F, D, ND = 16384, 26, 32, 13
K1, H1, H2, H3 = 896, 1024, 512, 256
K2, K3 = 1024, 512            # layers 2 / 3 K (bias vectors)
W = 36                        # sparse row: 32 emb + wide + pad (fp32 in the table)


def gemm(M, N, K, out_bytes, split=1):
    flops = 2.0 * M * N * K
    byts = (M * K + N * K) * 2 + M * N * out_bytes * split
    return flops, byts


def _split(n_out, k_in, blocks=256, min_rows=1024):
    """ops.linear_wgrad's split-K choice for W&D's overlapped weight gradients (blocks=256)."""
    tiles = ((n_out + 127) // 128) * ((k_in + 127) // 128)
    return max(1, min(B // min_rows, (blocks + tiles - 1) // tiles))


def spec(U):
    """(name regex, occurrence in the step, label, flops, bytes): the k-th kernel of the step (by
    start time) whose name matches -- kernels of one name keep their issue order across streams."""
    n = B * F
    s1, s2, s3 = _split(H1, K1), _split(H2, K2), _split(H3, K3)
    return [
        (r"gemm_v2_kernel<256, 256, false, false", 0, "fwd1 X.W1^T 16384x1024x896 +bias/ReLU", *gemm(B, H1, K1, 2)),
        (r"gemm_v2_kernel<128, 128, false, false", 0, f"fwd2 16384x512x{K2} +bias/ReLU", *gemm(B, H2, K2, 2)),
        (r"gemm_v2_kernel<128, 128, false, false", 1, f"fwd3 16384x256x{K3} +bias/ReLU", *gemm(B, H3, K3, 2)),
        (r"gemm_v2_kernel<128, 128, false, true", 0, "dgrad dH2 16384x512x256 (ReLU mask)",
         gemm(B, H2, H3, 2)[0], gemm(B, H2, H3, 2)[1] + B * H2 * 2),
        (r"gemm_v2_kernel<256, 256, false, true, 5", 0, "dgrad dH1 16384x1024x512 (ReLU mask)",
         gemm(B, H1, H2, 2)[0], gemm(B, H1, H2, 2)[1] + B * H1 * 2),
        (r"gemm_v2_kernel<256, 256, false, true, 4", 0, "dgrad dX 16384x832x1024", *gemm(B, F * D, H1, 2)),
        (r"gemm_v2_kernel<\d+, \d+, true, true", 0, f"wgrad W3 256x{K3}x16384 ({s3} split-K slabs)",
         *gemm(H3, K3, B, 4, s3)),
        (r"gemm_v2_kernel<\d+, \d+, true, true", 1, f"wgrad W2 512x{K2}x16384 ({s2} split-K slabs)",
         *gemm(H2, K2, B, 4, s2)),
        (r"gemm_v2_kernel<\d+, \d+, true, true", 2, f"wgrad W1 1024x896x16384 ({s1} split-K slabs)",
         *gemm(H1, K1, B, 4, s1)),
        (r"splitk_reduce_kernel", 0, f"split-K reduce W3 ({s3} planes)", 0, s3 * H3 * K3 * 4 + 2 * H3 * K3 * 4),
        (r"splitk_reduce_kernel", 1, f"split-K reduce W2 ({s2} planes)", 0, s2 * H2 * K2 * 4 + 2 * H2 * K2 * 4),
        (r"splitk_reduce_kernel", 2, f"split-K reduce W1 ({s1} planes)", 0, s1 * H1 * K1 * 4 + 2 * H1 * K1 * 4),
        (r"wd_assemble_tab_kernel", 0, "Get + assemble X (rows read from the fp32 shard + dense + wide sum)", 0,
         B * K1 * 2 + n * (D * 4 + 4 + 8 + 8) + B * ND * 4 + B * 4),
        (r"wd_head_kernel", 0, "head Linear 256->1 + BCE fwd/bwd (+ per-block dH3 column sums)", 0,
         B * H3 * 2 * 2 + B * 12),
        (r"wd_head_fold_kernel", 0, "head batch sums folded (weight-gradient stream)", 0, 256 * (2 * H3 + 2) * 4),
        (r"colsum_bf16_kernel", 0, "layer-2 bias gradient (dH2 column sums)", 0, B * H2 * 2),
        (r"colsum_fold_kernel", 0, "layer-2 bias gradient: fold of the column-sum partials", 0, 0),
        (r"zero_rows_dev_kernel", 0, "zero grad rows", 0, U * W * 4),
        (r"emb_seg_det_kernel", 0, "embedding backward: deterministic segment sums (dX rows gathered by the CSR)", 0,
         n * (D * 2 + 8 + 4) + U * W * 4),
        (r"emb_seg_fix_kernel", 0, "embedding backward: rows cut by piece boundaries (partials)", 0,
         (n // 128) * 2 * (D + 4) * 4 * 2),
        (r"sparse_rowwise_adagrad_v4", 0, "row-wise Adagrad apply (U rows)", 0, U * (W * 4 * 3 + 8 + 8 + 8)),
        (r"adam_kernel", 0, f"Adam (dense 1.58M params, folds the {s1}+{s2}+{s3} wgrad slab planes)", 0,
         1582080 * (16 + 18) + 4 * (s1 * H1 * K1 + s2 * H2 * K2 + s3 * H3 * K3)),
        (r"criteo_synth_kernel", 0, "synthetic batch (planning stream)", 0, B * (F * 8 + ND * 4 + 4)),
        (r"plan_transpose_kernel", 0, "plan: keys -> column-major (planning)", 0, n * (8 + 4)),
        (r"plan_sort_col_kernel", 0, "plan: per-column LDS radix sort, 26 WGs (planning)", 0, n * (4 + 4 + 4) + U * 8),
        (r"plan_emit_kernel", 0, "plan: uniq / inv / lookup CSR (planning)", 0, n * (4 + 4 + 8 + 4 + 4) + U * 16),
    ]


def measure_unique(batches=20):
    """Average unique-key count U per batch of bench.py's synthetic Criteo data (needs the GPU)."""
    import os
    import sys

    import torch

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from minips_amd import ops
    from minips_amd.data.synthetic import CriteoSynth
    from minips_amd.models.widedeep import WideDeepConfig

    dev = torch.device("cuda", 0)
    cfg = WideDeepConfig()
    data = CriteoSynth(B, cards=cfg.cards, device=dev, seed=1)
    bounds = torch.tensor([0, sum(cfg.cards)], device=dev)
    us = []
    for _ in range(batches):
        _, keys, _ = data.next()
        us.append(int(ops.unique_bucketize_n(keys, bounds, keys.shape[1])[3].item()))
    print(f"U mean {sum(us) / len(us):.0f} over {batches} batches of {keys.numel()} lookups (min {min(us)}, "
          f"max {max(us)})")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace", nargs="?")
    ap.add_argument("--U", type=float, help="unique keys per batch (--measure-U prints it)")
    ap.add_argument("--measure-U", action="store_true", help="measure U on the GPU and exit")
    ap.add_argument("--skip", type=int, default=3, help="steps to skip")
    a = ap.parse_args()
    if a.measure_U:
        return measure_unique()
    if not a.trace or a.U is None:
        ap.error("trace and --U are required")
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # one step = from one Adam (the last kernel of a step) to the next
    starts = [i for i, r in enumerate(rows) if "adam_kernel" in r["Kernel_Name"]]
    steps = [rows[starts[i] + 1: starts[i + 1] + 1] for i in range(a.skip, len(starts) - 1)]
    specs = spec(a.U)
    per = {}
    for st in steps:
        seen = {}
        for r in st:
            name = r["Kernel_Name"]
            for pat, k, label, fl, by in specs:
                if re.search(pat, name):
                    if seen.get(pat, 0) == k:
                        per.setdefault(label, (fl, by, []))[2].append((int(r["End_Timestamp"]) -
                                                                      int(r["Start_Timestamp"])) / 1e3)
                        seen[pat] = k + 1
                        break
                    if seen.get(pat, 0) > k:
                        continue
    print(f"# W&D 1-GPU step: per-kernel achieved rates ({len(steps)} steady steps, U = {a.U:.0f})\n")
    print("| kernel | us (median) | GFLOP | MB | TFLOP/s | % bf16 peak | TB/s | % HBM peak |")
    print("|---|---|---|---|---|---|---|---|")
    tot = 0.0
    for _, _, label, _, _ in specs:  # (in spec order)
        if label not in per:
            continue
        fl, by, ds = per[label]
        us = statistics.median(ds)
        tot += us
        tf = fl / us / 1e6
        tb = by / us / 1e6
        print(f"| {label} | {us:.1f} | {fl / 1e9:.1f} | {by / 1e6:.1f} | {tf:.0f} | {100 * tf / PEAK_TF:.0f}% | "
              f"{tb:.2f} | {100 * tb / PEAK_TB:.0f}% |")
    print(f"\nSum of the listed kernels: {tot:.0f} us per step (the streams overlap: compute, weight-gradient "
          "side stream, planning stream).")


if __name__ == "__main__":
    main()
