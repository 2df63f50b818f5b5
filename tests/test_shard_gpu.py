"""The sharded path with the real device pass: 2 ranks (gloo for the count
exchange) sharing cuda:0 -- the box has one GPU -- each running the fused HIP
kernel on its row range. Shards, offsets and the root gather must equal the
oracle over the whole table."""
import os

import pytest
import torch.multiprocessing as mp

from test_shard_cpu import DENSE, N, PRED, PROJS, SCHEMA, _free_port, table

pytestmark = pytest.mark.gpu


def _worker(rank, world, port, dense, q):
    try:
        import torch
        import torch.distributed as dist

        from datafusion_amd.execution.expression import compile_scalar_expr
        from datafusion_amd.execution.shard import ShardedFilterProject, gather_to_root, shard_range
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        lo, hi = shard_range(N, rank, world)
        batch, _ = table(lo, hi, nullable=dense)
        pred = None if dense else compile_scalar_expr(None, PRED, SCHEMA)
        projs = [compile_scalar_expr(None, e, SCHEMA) for e in (DENSE if dense else PROJS)]
        res = ShardedFilterProject(pred, projs)(batch)
        full = gather_to_root(res, [c.data_type for c in res.columns], root=0)
        q.put((rank, res.row_offset, res.total_rows, [c.cpu().to_pylist() for c in res.columns],
               None if full is None else [c.cpu().to_pylist() for c in full]))
        dist.destroy_process_group()
    except Exception as e:
        import traceback
        q.put(("error", traceback.format_exc(), str(e)))


@pytest.mark.parametrize("dense", [False, True])
def test_sharded_device_pass_matches_oracle(dense):
    from oracle_ffi import oracle_filter_project
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, dense, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = sorted([q.get(timeout=110) for _ in range(2)], key=lambda o: o[0])
    for p in procs:
        p.join(30)
    errs = [o for o in out if o[0] == "error"]
    assert not errs, errs[0][1]
    batch, _ = table(nullable=dense)
    ref = [r.to_pylist() for _, r in oracle_filter_project(SCHEMA, batch, None if dense else PRED,
                                                             DENSE if dense else PROJS)]
    for rank, off, tot, shard, _ in out:
        assert tot == len(ref[0])
        for o in range(len(ref)):
            assert shard[o] == ref[o][off: off + len(shard[0])]
    assert out[0][4] == ref
