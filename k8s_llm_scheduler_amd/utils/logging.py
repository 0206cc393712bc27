"""Logging setup.

Reference: ``scheduler.py:26-41`` -- level from ``LOG_LEVEL``; ``LOG_FORMAT=json`` only switched
the format string to ``'%(message)s'`` (no actual JSON).  Here ``format: json`` emits one JSON
object per line (timestamp, level, logger, message, plus ``rank`` under torchrun), ``text`` keeps
the reference's ``'%(asctime)s - %(name)s - %(levelname)s - %(message)s'``, and ``logging.file``
(``config.yaml:26``, unused by the reference) adds a file handler.
"""

from __future__ import annotations

import json
import logging
import os
import time
from typing import Optional

TEXT_FORMAT = "%(asctime)s - %(name)s - %(levelname)s - %(message)s"


class JsonFormatter(logging.Formatter):
    def format(self, record: logging.LogRecord) -> str:
        d = {
            "ts": time.strftime("%Y-%m-%dT%H:%M:%S", time.gmtime(record.created)) + f".{int(record.msecs):03d}Z",
            "level": record.levelname,
            "logger": record.name,
            "message": record.getMessage().strip(),
        }
        if "RANK" in os.environ:
            d["rank"] = int(os.environ["RANK"])
        if record.exc_info:
            d["exc"] = self.formatException(record.exc_info)
        return json.dumps(d)


def setup_logging(level: str = "INFO", fmt: str = "text", file: Optional[str] = None) -> None:
    root = logging.getLogger()
    for h in list(root.handlers):
        root.removeHandler(h)
    formatter: logging.Formatter = JsonFormatter() if fmt == "json" else logging.Formatter(TEXT_FORMAT)
    handlers = [logging.StreamHandler()]
    if file:
        handlers.append(logging.FileHandler(file))
    for h in handlers:
        h.setFormatter(formatter)
        root.addHandler(h)
    root.setLevel(getattr(logging, str(level).upper(), logging.INFO))
