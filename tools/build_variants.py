#!/usr/bin/env python
"""Build diagnostic variants of libsem_hip.so for A/B timing on the GPU box:

  python tools/build_variants.py NAME:DEF1,DEF2 [NAME:...]

writes build_variants/NAME/libsem_hip.so compiled with -DDEF1 -DDEF2 (every
order; an entry starting with "-" is a raw compiler flag, e.g.
nolicm:-mllvm,-disable-machine-licm); select one at run time with
SEM_LIB_PATH=build_variants/NAME/libsem_hip.so."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from spectralelementmethod_amd import _build  # noqa: E402

for spec in sys.argv[1:]:
    name, _, defs = spec.partition(":")
    d = os.path.join(ROOT, "build_variants", name)
    os.makedirs(d, exist_ok=True)
    out = os.path.join(d, _build.LIB_NAME)
    _build.build(force=False, verbose=False, out=out, defines=[x for x in defs.split(",") if x])
    print("built", out, defs)
