"""Logging setup.  Mirrors the reference's levels (``appsettings.json:2-6``:
Default=Information, Microsoft.AspNetCore=Warning) and keeps its ``[RAG]`` message
prefixes (``Helpers/RagIndex.cs:18,29,33,52,55``)."""
from __future__ import annotations

import logging
import os
import sys

_configured = False


def setup(level: str | None = None):
    global _configured
    if _configured:
        return
    lvl = (level or os.environ.get("LK_LOG_LEVEL", "INFO")).upper()
    h = logging.StreamHandler(sys.stderr)
    h.setFormatter(logging.Formatter("%(asctime)s %(levelname)s %(name)s: %(message)s"))
    root = logging.getLogger("lk")
    root.addHandler(h)
    root.setLevel(getattr(logging, lvl, logging.INFO))
    root.propagate = False
    for noisy in ("uvicorn.access", "httpx"):
        logging.getLogger(noisy).setLevel(logging.WARNING)
    _configured = True


def get_logger(name: str) -> logging.Logger:
    setup()
    return logging.getLogger("lk." + name)
