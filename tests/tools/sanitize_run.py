#!/usr/bin/env python3
"""Run CPU tests against the ASan + UBSan builds of the checker (oracle/_build/librt_oracle_asan.so)
and of the host runtime (gpgpuraytrace_amd/_build/librt_hip_asan.so).  Started by
scripts/sanitize_cpu.sh, which preloads the sanitizer runtime; pytest arguments pass through."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import oracle_lib  # noqa: E402
import with_variant  # noqa: E402

oracle_lib.LIB_PATH = os.path.join(ROOT, "oracle", "_build", "librt_oracle_asan.so")
with_variant.apply("asan")

import pytest  # noqa: E402

sys.exit(pytest.main(sys.argv[1:]))
