#!/usr/bin/env python3
"""Experiment builds of libchunkfs_amd.so with compile-time scan variants, each
into _exp/<name>/ (git-ignored; travels with the gpurun snapshot).  Select one
at run time with CHUNKFS_AMD_LIB=_exp/<name>/lib.so.  Diagnostics only.
Usage: python3 tools/build_variants.py name=DEF1,DEF2 ..."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from chunkfs_amd import build  # noqa: E402

for arg in sys.argv[1:]:
    name, _, defs = arg.partition("=")
    d = os.path.join(ROOT, "_exp", name)
    build.build(defines=[x for x in defs.split(",") if x], lib=os.path.join(d, "lib.so"), build_dir=d)
