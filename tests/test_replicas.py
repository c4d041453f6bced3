"""The N>1 bench path (independent replicas, one process per GPU) on CPU with gloo, world size 2."""
import os
import socket
import time

import pytest

torch = pytest.importorskip("torch")
import torch.multiprocessing as mp  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    from graphslam_amd.replicas import init_from_env, timed_steps
    r = init_from_env()
    calls = []

    def step():
        time.sleep(0.05 * (r.rank + 1))     # rank 1 is the slow one
        calls.append(1)
        return 3 + r.rank, {"rank": r.rank}

    elapsed, units, results = timed_steps(r, step, steps=4, warmup=2)
    q.put((r.rank, elapsed, units, len(calls), results[-1][1]["rank"]))
    r.close()


def test_replicas_gloo_world2():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(k, world, port, q)) for k in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    out.sort()
    # both ranks agree on the max-over-ranks time, which is the slow rank's (4 x 0.1 s)
    assert abs(out[0][1] - out[1][1]) < 1e-12
    assert 0.38 < out[0][1] < 2.0
    # work summed over ranks: 4 steps x (3 + 4)
    assert out[0][2] == out[1][2] == 28
    # warmup calls are untimed but executed
    assert out[0][3] == out[1][3] == 6
    assert [o[4] for o in out] == [0, 1]
