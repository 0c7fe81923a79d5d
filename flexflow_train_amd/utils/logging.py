"""Logger categories (reference: lib/runtime/src/loggers.cc:4-8 — profile,
measure, sim, ps_sim, xfer_sim, xfer_est, metrics, Model, Mapper — and the
Python flexflow_logger).  Standard ``logging`` loggers under "flexflow.*";
the level comes from ``FF_LOG_LEVEL`` (e.g. ``debug``) or
``FF_LOG_LEVEL_<CATEGORY>``; every record carries the rank so interleaved
multi-process output stays readable."""
from __future__ import annotations

import logging
import os

CATEGORIES = ("profile", "measure", "sim", "search", "comm", "metrics", "model", "mapper", "runtime", "kernels")

_configured = False


class _RankFilter(logging.Filter):
    def filter(self, record):
        record.rank = os.environ.get("RANK", "0")
        return True


def _configure():
    global _configured
    if _configured:
        return
    _configured = True
    root = logging.getLogger("flexflow")
    h = logging.StreamHandler()
    h.setFormatter(logging.Formatter("[%(rank)s] %(name)s %(levelname)s: %(message)s"))
    h.addFilter(_RankFilter())
    root.addHandler(h)
    root.propagate = False
    root.setLevel(os.environ.get("FF_LOG_LEVEL", "WARNING").upper())


def get_logger(category: str) -> logging.Logger:
    _configure()
    lg = logging.getLogger(f"flexflow.{category}")
    lvl = os.environ.get(f"FF_LOG_LEVEL_{category.upper()}")
    if lvl:
        lg.setLevel(lvl.upper())
    return lg
