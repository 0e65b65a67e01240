#!/usr/bin/env python3
"""Run bench.py with Python-level settings applied first (A/B of host-side variants within one call).
usage: ab_py.py "<python statements>" [bench args...]   e.g. ab_py.py "IndexCorpus._count_read = 'copy'" --no-cpu"""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hilbert-quantization_amd")]
from hq_mi355x.core import search_engine  # noqa: E402
from hq_mi355x.core.search_engine import IndexCorpus  # noqa: E402,F401

exec(sys.argv[1])
sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[2:]
runpy.run_path(sys.argv[0], run_name="__main__")
