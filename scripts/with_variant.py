#!/usr/bin/env python3
"""Run a Python program (or -m module) against an EXPERIMENT build of the library.

    RT_LIB_VARIANT=<name> python3 scripts/with_variant.py bench.py --steps 12 ...
    RT_LIB_VARIANT=<name> python3 scripts/with_variant.py -m pytest tests -m gpu ...

loads gpgpuraytrace_amd/_build/librt_hip_<name>.so (make -C gpgpuraytrace_amd/csrc variant NAME=<name>
FLAGS=..., or `make trace`) in place of librt_hip.so; an empty or unset RT_LIB_VARIANT keeps the
default build.  Diagnostics only: the package itself reads no environment variable.
"""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def apply(name=None):
    """Point the package's loader at librt_hip_<name>.so (before its first lib() call)."""
    from gpgpuraytrace_amd import _native
    name = os.environ.get("RT_LIB_VARIANT", "") if name is None else name
    if name:
        if _native._lib is not None:
            raise RuntimeError("with_variant.apply: the default library is already loaded")
        _native.LIB_PATH = os.path.join(_native.HERE, "_build", f"librt_hip_{name}.so")
    return _native.LIB_PATH


if __name__ == "__main__":
    apply()
    args = sys.argv[1:]
    if not args:
        sys.exit(__doc__)
    if args[0] == "-m":
        sys.argv = [args[1]] + args[2:]
        runpy.run_module(args[1], run_name="__main__", alter_sys=True)
    else:
        sys.argv = args
        sys.path.insert(0, os.path.dirname(os.path.abspath(args[0])))
        runpy.run_path(args[0], run_name="__main__")
