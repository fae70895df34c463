"""Self-launch of one process per GPU (what `torch.distributed.run --nproc-per-node N` does for the
driver's N > 1 runs), so `python bench.py --gpus N` measures N ranks when started by hand too.

The parent never touches the GPU (no HIP call before or after the fork: each rank is a fresh
`python` child started with subprocess, never an exec of this process).  Each child gets RANK /
LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT in its environment; the parent waits
for all of them, stops the rest (by their own PIDs) as soon as one fails, and returns the first
non-zero exit code (0 when every rank succeeded).
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys
import time
from typing import List, Optional, Sequence


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def is_rank_process() -> bool:
    return "WORLD_SIZE" in os.environ


def spawn(n: int, cmd: Sequence[str], timeout: Optional[float] = None, extra_env: Optional[dict] = None) -> int:
    """Run `cmd` as n rank processes; returns the first non-zero exit code, else 0."""
    port = free_port()
    procs: List[subprocess.Popen] = []
    for r in range(n):
        env = dict(os.environ)
        env.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC for RCCL (the box's host driver)
        if extra_env:
            env.update(extra_env)
        procs.append(subprocess.Popen(list(cmd), env=env))
    t0 = time.time()
    rc = 0
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad and rc == 0:
                rc = bad[0]
                break
            if all(c is not None for c in codes):
                break
            if timeout is not None and time.time() - t0 > timeout:
                rc = 124
                break
            time.sleep(0.2)
    finally:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    return rc


def maybe_spawn(n: int, argv: Optional[Sequence[str]] = None) -> Optional[int]:
    """If n > 1 and this process is not a rank yet, start n ranks of this same command line and
    return their exit code (the caller exits with it); else None (run in this process)."""
    if n <= 1 or is_rank_process():
        return None
    argv = list(sys.argv if argv is None else argv)
    return spawn(n, [sys.executable] + argv)
