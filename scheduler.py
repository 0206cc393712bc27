#!/usr/bin/env python3
"""Drop-in entry point: ``python scheduler.py`` starts the scheduler like the reference's
``scheduler.py`` (same config.yaml, same schedulerName), with the decision LLM running locally on
MI355X.  Multi-GPU: ``torchrun --nproc-per-node 8 --master-addr 127.0.0.1 scheduler.py``.
See ``python -m k8s_llm_scheduler_amd --help`` for the other commands (verify, smoke)."""

import sys

from k8s_llm_scheduler_amd.__main__ import main

if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
