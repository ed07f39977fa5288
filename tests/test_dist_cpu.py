"""Multi-process (world size 2) CPU test of the N > 1 path: bench.py's clip
sharding, the TCP rendezvous that carries the RCCL unique id / barrier /
max-over-ranks timing, and the gather of token ids — compared with gloo's
gather and with a single-process run over the whole batch.  The GPU data
path replaces the gather with ncclGather over xGMI (wmi_dist_gather_tokens)."""
import json
import os
import socket
import subprocess
import sys

import numpy as np

from conftest import ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_rank_shard_and_gather(micro_model):
    world, cpg, n_tok = 2, 2, 6
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), OMP_NUM_THREADS="1")
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "dist_worker.py"), micro_model,
                                       str(cpg), str(n_tok)], env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                                      text=True))
    outs = [p.communicate(timeout=300) for p in procs]
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, e[-2000:]
    res = json.loads(outs[0][0].strip().splitlines()[-1])
    assert res["uid"] == "uid-from-rank0"
    assert res["tmax"] == 2.0
    tcp = np.array(res["tcp"])
    gloo = np.array(res["gloo"])
    assert tcp.shape == (world, cpg, n_tok)
    np.testing.assert_array_equal(tcp, gloo)
    # single process over the whole batch, clip c <- seed 1234 + c
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import dist_worker
    full = np.concatenate([dist_worker.decode_shard(micro_model, r, cpg, n_tok) for r in range(world)])
    np.testing.assert_array_equal(tcp.reshape(world * cpg, n_tok), full)
