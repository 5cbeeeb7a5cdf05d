#!/usr/bin/env python3
"""Diagnostic: run the word-tile pack of tests/test_gpu_wordtiles.py's kind-2
batch through a WT_CHECK build (prints state mismatches from the kernel)."""
import ctypes as C, os, random, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "capnproto-rust_amd")); sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch
import oracle_lib as O
from capnp_amd import _lib
_lib.LIB_PATH = os.path.abspath(sys.argv[1])  # (the diagnostic build, before the first load)
import test_gpu_wordtiles as T
rng = random.Random(202)
sizes = T._sizes_long(rng, 300)
offs = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
words = O.gen_fill(offs, kind0=2, pz=O.PZ30, id0=2 * 77)
from capnp_amd import Context
ctx = Context(0)
try:
    T._check_pack(ctx, words, offs)
    print("ok")
except AssertionError as e:
    print("mismatch", str(e)[:200])
torch.cuda.synchronize()
