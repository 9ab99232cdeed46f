"""stdout + file logging in the reference's line format (utils/logger.py:9-58)."""
from __future__ import annotations

import logging
import os

from .utils import get_local_time

_LEVELS = {"info": logging.INFO, "debug": logging.DEBUG, "error": logging.ERROR,
           "warning": logging.WARNING, "critical": logging.CRITICAL}


def init_logger(config) -> None:
    root = config["log_root"] or "./log/"
    os.makedirs(os.path.dirname(root) or ".", exist_ok=True)
    os.makedirs(root, exist_ok=True)
    path = os.path.join(root, "{}-{}-{}.log".format(config["model"], config["dataset"], get_local_time()))
    level = _LEVELS.get((config["state"] or "info").lower(), logging.INFO)
    fh = logging.FileHandler(path, "w", "utf-8")
    fh.setLevel(level)
    fh.setFormatter(logging.Formatter("%(asctime)-15s %(levelname)s %(message)s", "%a %d %b %Y %H:%M:%S"))
    sh = logging.StreamHandler()
    sh.setLevel(level)
    sh.setFormatter(logging.Formatter("%(asctime)-15s %(levelname)s %(message)s", "%d %b %H:%M"))
    logging.basicConfig(level=level, handlers=[sh, fh], force=True)
