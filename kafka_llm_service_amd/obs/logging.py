"""Structured logging (SURVEY.md §5.5 "structured JSON logs"; the reference used ~127 emoji print() calls).

``setup_logging()`` installs one handler on the ``kafka`` logger tree: plain ``time level logger message`` lines by
default, one JSON object per line with ``KAFKA_LOG_JSON=1`` (ts, level, logger, msg, pid, thread, exception and any
``extra=`` fields), level from ``KAFKA_LOG_LEVEL`` (default INFO).
"""
from __future__ import annotations

import json
import logging
import os
import sys
import time

_STD = set(vars(logging.makeLogRecord({})).keys()) | {"message", "asctime"}


class JsonFormatter(logging.Formatter):
    def format(self, record: logging.LogRecord) -> str:
        d = {"ts": round(record.created, 6), "time": time.strftime("%Y-%m-%dT%H:%M:%S", time.gmtime(record.created)),
             "level": record.levelname, "logger": record.name, "msg": record.getMessage(), "pid": record.process,
             "thread": record.threadName}
        for k, v in record.__dict__.items():
            if k not in _STD and not k.startswith("_"):
                try:
                    json.dumps(v)
                    d[k] = v
                except TypeError:
                    d[k] = repr(v)
        if record.exc_info:
            d["exc"] = self.formatException(record.exc_info)
        return json.dumps(d, ensure_ascii=False)


def setup_logging(json_lines: bool | None = None, level: str | None = None, stream=None) -> logging.Logger:
    json_lines = os.environ.get("KAFKA_LOG_JSON", "0") == "1" if json_lines is None else json_lines
    level = level or os.environ.get("KAFKA_LOG_LEVEL", "INFO")
    root = logging.getLogger("kafka")
    for h in list(root.handlers):
        if getattr(h, "_kafka", False):
            root.removeHandler(h)
    h = logging.StreamHandler(stream or sys.stderr)
    h._kafka = True
    h.setFormatter(JsonFormatter() if json_lines else
                   logging.Formatter("%(asctime)s %(levelname)s %(name)s: %(message)s"))
    root.addHandler(h)
    root.setLevel(level.upper())
    root.propagate = False
    return root
