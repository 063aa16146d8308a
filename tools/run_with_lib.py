#!/usr/bin/env python3
"""Run a Python tool against an alternate libzcrc build (same-box A/B of two
builds; measurement tooling).   python tools/run_with_lib.py LIB SCRIPT [args]"""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import zipsfs_amd._lib as L  # noqa: E402

L.LIB_PATH = os.path.abspath(sys.argv[1])
sys.argv = sys.argv[2:]
sys.path.insert(0, os.path.dirname(os.path.abspath(sys.argv[0])))
runpy.run_path(sys.argv[0], run_name="__main__")
