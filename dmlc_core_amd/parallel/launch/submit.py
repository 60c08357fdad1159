"""dmlc-submit entry point (reference `tracker/dmlc_tracker/submit.py:13-56`).

    python -m dmlc_core_amd.parallel.launch.submit --cluster local --num-workers 8 \
        --gpus-per-node 8 --torch-env 1 python train.py

Backends are imported lazily (the reference hard-imported ``kubernetes`` and
failed without it, §7.4 #6); every choice accepted by the parser is wired
(the reference accepted ssh/slurm but never dispatched them).
"""
from __future__ import annotations

import importlib
import logging
import sys

from .opts import get_opts


def config_logger(args) -> None:
    fmt = "%(asctime)s %(levelname)s %(message)s"
    level = getattr(logging, args.log_level)
    if args.log_file is None:
        logging.basicConfig(format=fmt, level=level)
    else:
        logging.basicConfig(format=fmt, level=level, filename=args.log_file)
        console = logging.StreamHandler()
        console.setFormatter(logging.Formatter(fmt))
        console.setLevel(level)
        logging.getLogger("").addHandler(console)


def main(argv=None) -> int:
    args = get_opts(argv)
    config_logger(args)
    backend = importlib.import_module(f"dmlc_core_amd.parallel.launch.{args.cluster}")
    return backend.submit(args) or 0


if __name__ == "__main__":
    sys.exit(main())
