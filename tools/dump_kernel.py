#!/usr/bin/env python3
"""Write the generated query kernel of a bench configuration to a .hip file
(for hipcc -Rpass-analysis=kernel-resource-usage / ISA inspection).
usage: tools/dump_kernel.py c2|c4 out.hip"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from test_jit_cpu import F3, c2_query, jit_check  # noqa: E402


def main():
    which, out = sys.argv[1], sys.argv[2]
    if which == "c2":
        pred, projs = c2_query()
        rc, code, msg, src = jit_check(F3, pred, projs)
    else:
        raise SystemExit("unknown config")
    assert rc > 0, msg
    src = src.replace('extern "C" __global__', 'extern "C" __global__ __attribute__((used))')
    open(out, "w").write('#include <hip/hip_runtime.h>\n' + src)


if __name__ == "__main__":
    main()
