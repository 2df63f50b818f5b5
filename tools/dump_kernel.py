#!/usr/bin/env python3
"""Write the generated query kernel of a bench configuration to a .hip file
(for hipcc -Rpass-analysis=kernel-resource-usage / ISA inspection).
usage: tools/dump_kernel.py c2|c3eq|c3lt[b] out.hip  (suffix b: the coalesced-batches form)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from test_jit_cpu import F3, c2_query, jit_check  # noqa: E402
from datafusion_amd.arrow import Field, Schema  # noqa: E402
from datafusion_amd.logicalplan import BinaryExpr, Column, DataType, Float64, Literal, Operator, Utf8  # noqa: E402

C3 = Schema([Field("s", DataType.Utf8, False), Field("v", DataType.Float64, True)])


def main():
    which, out = sys.argv[1], sys.argv[2]
    bflag = 0x40000000 if which.endswith("b") else 0
    which = which.rstrip("b")
    if which == "c2":
        pred, projs = c2_query()
        rc, code, msg, src = jit_check(F3, pred, projs, flags=bflag)
    elif which in ("c3eq", "c3lt"):
        pred = (BinaryExpr(Column(0), Operator.Eq, Literal(Utf8("w17dizjxms"))) if which == "c3eq"
                else BinaryExpr(Column(1), Operator.Lt, Literal(Float64(0.5))))
        rc, code, msg, src = jit_check(C3, pred, [Column(0), Column(1)], flags=2 | bflag)
    else:
        raise SystemExit("unknown config")
    assert rc > 0, msg
    src = src.replace('extern "C" __global__', 'extern "C" __global__ __attribute__((used))')
    open(out, "w").write('#include <hip/hip_runtime.h>\n' + src)


if __name__ == "__main__":
    main()
