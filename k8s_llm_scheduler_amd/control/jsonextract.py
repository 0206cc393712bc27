"""Extract the decision JSON object from model output text.

Same three strategies, in the same order, as the reference ``_extract_json``
(``scheduler.py:474-519``):

1. the text between the first "```json" fence and the next "```",
2. the object starting at the **last** ``{`` (brace-matched),
3. the object starting at the **first** ``{`` (brace-matched).

The brace matcher is the reference's naive counter (braces inside JSON strings are counted), and
for strategies 2 and 3 every balanced close is tried in turn, exactly as the reference loop
does (it keeps scanning after a failed ``json.loads``).  Returns a ``dict`` or ``None``; a
non-object JSON value in the fence is returned as-is, like the reference.
"""

from __future__ import annotations

import json
from typing import Any, Optional


def _scan_from(text: str, start: int) -> Optional[Any]:
    depth = 0
    for i in range(start, len(text)):
        ch = text[i]
        if ch == "{":
            depth += 1
        elif ch == "}":
            depth -= 1
            if depth == 0:
                try:
                    return json.loads(text[start:i + 1])
                except json.JSONDecodeError:
                    pass
    return None


def extract_json(text: str) -> Optional[Any]:
    if text is None:
        return None
    fence = text.find("```json")
    if fence != -1:
        begin = fence + 7
        end = text.find("```", begin)
        if end != -1:
            try:
                return json.loads(text[begin:end].strip())
            except json.JSONDecodeError:
                pass
    last = text.rfind("{")
    if last != -1:
        got = _scan_from(text, last)
        if got is not None:
            return got
    first = text.find("{")
    if first != -1:
        got = _scan_from(text, first)
        if got is not None:
            return got
    return None


def json_object_closed(text: str) -> bool:
    """Cheap streaming stop test used by the engine: True once the first top-level ``{`` in the
    text has been balanced by a ``}`` (naive counter, same as above)."""
    start = text.find("{")
    if start == -1:
        return False
    depth = 0
    for ch in text[start:]:
        if ch == "{":
            depth += 1
        elif ch == "}":
            depth -= 1
            if depth == 0:
                return True
    return False
