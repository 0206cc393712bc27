#!/usr/bin/env python3
"""Merge the rows of `tools/mgemm_tune.py --json-out` runs into the mgemm plan table
(engine/assets/mgemm_gfx950.json), e.g. after a tuning run on a GPU box whose own table copy is not kept.

    python tools/mgemm_table_merge.py gpurun_out/r20/small_m_bf16.json gpurun_out/r20/fp8.json
"""

from __future__ import annotations

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from k8s_llm_scheduler_amd import ops  # noqa: E402


def main(paths) -> int:
    with open(ops.MG_TABLE_PATH) as f:
        table = json.load(f)
    n = 0
    for p in paths:
        with open(p) as f:
            rows = json.load(f)
        for r in rows:
            key = f"{ops._mg_bucket(r['M'])},{r['N']},{r['K']},{r['epi']},{int(bool(r['fp8']))}"
            table["plans"][key] = [r["cfg"], r["grid"], r["mgemm_us"], r["lib_us"]]
            n += 1
    with open(ops.MG_TABLE_PATH, "w") as f:
        json.dump(table, f, indent=0, sort_keys=True)
    print(f"merged {n} rows; table has {len(table['plans'])} plans")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
