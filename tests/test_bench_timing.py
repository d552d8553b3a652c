"""bench.py's timed bracket at world 2 on gloo (CPU): a step holding a collective — as the N>1 C3
step does (kd_diff2_gather) — must run the same number of times on every rank, the pre-timing burst
included, even when the ranks' steps take different times."""
import os
import socket
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class _Eng:
    def sync(self):
        pass

    def device_sync(self):
        pass


def _worker(rank, world, port, out_dir):
    import time

    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank))
    sys.path.insert(0, ROOT)
    import bench

    H = bench.Harness()
    try:
        calls = [0]

        def step():  # rank 1's steps are 3x slower; each step all-reduces (a mismatched count hangs)
            time.sleep(0.002 * (1 + 2 * rank))
            t = torch.ones(1)
            dist.all_reduce(t)
            calls[0] += 1

        sec = bench.timed(H, _Eng(), step, 5)
        np.save(os.path.join(out_dir, f"r{rank}.npy"), np.array([calls[0], sec]))
    finally:
        H.close()


def test_timed_same_step_count_on_every_rank(tmp_path):
    import torch.multiprocessing as mp

    mp.start_processes(_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True, start_method="spawn")
    r0, r1 = np.load(tmp_path / "r0.npy"), np.load(tmp_path / "r1.npy")
    assert r0[0] == r1[0] and r0[0] > 5  # the burst ran, the same number of steps on both ranks
    assert r0[1] == r1[1]  # the max over ranks
