#!/usr/bin/env python3
"""Per-kernel breakdown of the LAST prefill forward (and the last decode step) in a rocprofv3 kernel trace.

rocprofv3 --stats averages every call of a kernel over the whole run, including start-up graph captures at other row
counts; this reads the per-dispatch trace (``*kernel_trace.csv``) instead and isolates the last forward of the run:

* prefill: the contiguous run of dispatches that ends with the last prefill-attention / big-GEMM kernel, back to the
  decode GEMV that precedes it;
* decode: the dispatches between the last two embedding kernels, plus a per-layer view: the kernels of one decoder
  layer in launch order (the period between decode-attention launches), each averaged over the middle layers, so
  projections that share a kernel template (O and down) are told apart.

    python tools/last_forward.py <kernel_trace.csv>
"""

import csv
import sys
from collections import defaultdict

PREFILL_MARK = ("paged_prefill_kernel", "pgemm_kernel", "pgemm4_kernel", "pgemm_reduce", "rope_kv_kernel",
                "Cijk_", "quantize_act_fp8")


def short(name: str) -> str:
    n = name.split("(")[0]
    return n.replace("void ", "").replace("k8sllm::", "")[:90]


def table(rows, title):
    if not rows:
        print(f"== {title}: none")
        return
    span = (rows[-1][2] - rows[0][1]) / 1e3
    busy = sum(e - s for _, s, e in rows) / 1e3
    per = defaultdict(lambda: [0, 0.0])
    for n, s, e in rows:
        per[short(n)][0] += 1
        per[short(n)][1] += (e - s) / 1e3
    print(f"== {title}: {len(rows)} dispatches, span {span:.1f} us, kernel busy {busy:.1f} us, gaps {span - busy:.1f} us")
    for n, (c, t) in sorted(per.items(), key=lambda kv: -kv[1][1]):
        print(f"{t:10.1f} us {c:6d} x {t / c:8.2f} us  {n}")


def main() -> int:
    rows = []
    with open(sys.argv[1]) as f:
        for r in csv.DictReader(f):
            name = r.get("Kernel_Name") or r.get("KernelName") or r.get("Name")
            s = int(r.get("Start_Timestamp") or r.get("BeginNs") or r["Start"])
            e = int(r.get("End_Timestamp") or r.get("EndNs") or r["End"])
            rows.append((name, s, e))
    rows.sort(key=lambda t: t[1])
    is_pf = [any(m in n for m in PREFILL_MARK) for n, _, _ in rows]
    last = max((i for i, p in enumerate(is_pf) if p), default=None)
    if last is not None:
        # walk back to the embedding that starts this forward (prefill forwards begin with one)
        first = last
        while first > 0 and "embedding_kernel" not in rows[first][0]:
            first -= 1
        end = last
        while end + 1 < len(rows) and not rows[end + 1][0].startswith(("void k8sllm::gemv", "k8sllm::embedding")) \
                and "sample" not in rows[end][0]:
            end += 1
        table(rows[first:end + 1], "last prefill forward")
    emb = [i for i, (n, _, _) in enumerate(rows) if "embedding_kernel" in n]
    if len(emb) >= 2:
        table(rows[emb[-2]:emb[-1]], "last decode step")
        layer_view(rows[emb[-2]:emb[-1]])
    return 0


def layer_view(rows) -> None:
    att = [i for i, (n, _, _) in enumerate(rows)
           if any(k in n for k in ("decode_fused", "decode_split", "paged_decode"))]
    if len(att) < 4:
        return
    per = att[1] - att[0]
    if any(b - a != per for a, b in zip(att, att[1:])):
        return
    mid = att[1:-1]                 # layers with a full period on both sides
    print(f"== per-layer view of the last decode step: {per} kernels per layer, mean over {len(mid)} layers "
          f"(offsets from the attention launch)")
    tot = 0.0
    for off in range(-1, per - 1):
        d = [(rows[i + off][2] - rows[i + off][1]) / 1e3 for i in mid if 0 <= i + off < len(rows)]
        gap = [(rows[i + off][1] - rows[i + off - 1][2]) / 1e3 for i in mid if 1 <= i + off < len(rows)]
        tot += sum(d) / len(d)
        print(f"  {off:+d} {sum(d) / len(d):8.2f} us (gap before {sum(gap) / len(gap):5.2f})  {short(rows[mid[0] + off][0])}")
    print(f"  layer kernel time {tot:.2f} us")


if __name__ == "__main__":
    sys.exit(main())
