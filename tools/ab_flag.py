#!/usr/bin/env python
"""Run bench.py with one engine module flag overridden (in-process A/B of a Python-side
structure switch).  usage: python tools/ab_flag.py NAME=VALUE [bench.py args...]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
name, val = sys.argv[1].split("=")
from savqa_amd import engine  # noqa: E402

setattr(engine, name, type(getattr(engine, name))(eval(val)))
sys.argv = ["bench.py"] + sys.argv[2:]
import bench  # noqa: E402

bench.main()
