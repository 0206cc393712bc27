"""Kubernetes resource-quantity parsing.

Two modes:

``reference`` reproduces the reference exactly, quirks included:
  * node side (``scheduler.py:172-187``): cpu ``"Nm"`` -> N/1000 else ``float``; memory
    ``Ki``/``Mi``/``Gi`` else bytes / 1024**3.  Anything else raises ``ValueError`` (which makes
    the reference's snapshot return ``[]``, ``scheduler.py:168-170``).
  * pod side (``scheduler.py:742-753``): cpu like the node side; memory only ``Ki``/``Mi``/``Gi``
    contribute, any other suffix or a plain byte count contributes **0**.

``full`` accepts every Kubernetes quantity form (decimal SI ``n u m k M G T P E``, binary
``Ki Mi Gi Ti Pi Ei``, exponent ``1e3``) and agrees with ``reference`` on every input the
reference accepts on the node side.  It is the default (config ``compat.quantity_parsing``)
because the reference's failure modes (no schedulable nodes / free memory) break scheduling.
"""

from __future__ import annotations

import re
from typing import Any

_BIN = {"Ki": 2 ** 10, "Mi": 2 ** 20, "Gi": 2 ** 30, "Ti": 2 ** 40, "Pi": 2 ** 50, "Ei": 2 ** 60}
_DEC = {"n": 1e-9, "u": 1e-6, "m": 1e-3, "": 1.0, "k": 1e3, "M": 1e6, "G": 1e9, "T": 1e12,
        "P": 1e15, "E": 1e18}
_QTY = re.compile(r"^\s*([+-]?(?:\d+\.?\d*|\.\d+)(?:[eE][+-]?\d+)?)\s*(Ki|Mi|Gi|Ti|Pi|Ei|[numkMGTPE]?)\s*$")
_GIB = float(2 ** 30)


def parse_quantity(q: Any) -> float:
    """Parse a Kubernetes quantity to a float in base units (cores / bytes)."""
    if isinstance(q, (int, float)):
        return float(q)
    m = _QTY.match(str(q))
    if not m:
        raise ValueError(f"invalid quantity: {q!r}")
    num, suf = float(m.group(1)), m.group(2)
    return num * (_BIN[suf] if suf in _BIN else _DEC[suf])


# ---------------------------------------------------------------- node side (allocatable)
def node_cpu(s: Any, mode: str = "full") -> float:
    if mode == "reference":
        s = str(s)
        return float(s[:-1]) / 1000 if s.endswith("m") else float(s)
    return parse_quantity(s)


def node_memory_gb(s: Any, mode: str = "full") -> float:
    if mode == "reference":
        s = str(s)
        if s.endswith("Ki"):
            return float(s[:-2]) / 1024 / 1024
        if s.endswith("Mi"):
            return float(s[:-2]) / 1024
        if s.endswith("Gi"):
            return float(s[:-2])
        return float(s) / 1024 / 1024 / 1024
    # Same arithmetic order as the reference for Ki/Mi/Gi so values are bit-identical.
    m = _QTY.match(str(s)) if not isinstance(s, (int, float)) else None
    if m and m.group(2) == "Ki":
        return float(m.group(1)) / 1024 / 1024
    if m and m.group(2) == "Mi":
        return float(m.group(1)) / 1024
    if m and m.group(2) == "Gi":
        return float(m.group(1))
    return parse_quantity(s) / 1024 / 1024 / 1024


# ---------------------------------------------------------------- pod side (requests)
def pod_cpu(s: Any, mode: str = "full") -> float:
    if mode == "reference":
        if isinstance(s, str) and s.endswith("m"):
            return float(s[:-1]) / 1000
        return float(s or 0)
    if s is None or s == "":
        return 0.0
    if isinstance(s, str) and s.endswith("m"):
        return float(s[:-1]) / 1000
    return parse_quantity(s)


def pod_memory_gb(s: Any, mode: str = "full") -> float:
    if mode == "reference":
        if isinstance(s, str):
            if s.endswith("Ki"):
                return float(s[:-2]) / 1024 / 1024
            if s.endswith("Mi"):
                return float(s[:-2]) / 1024
            if s.endswith("Gi"):
                return float(s[:-2])
        return 0.0
    if s is None or s == "":
        return 0.0
    return node_memory_gb(s, "full")
