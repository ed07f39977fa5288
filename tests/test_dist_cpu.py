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
import time

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


def test_bench_launches_its_own_ranks():
    """`python3 bench.py --gpus 2` without torchrun's environment starts its two
    rank processes itself (configs[3]'s 8 clips per GPU by default), they meet
    over the TCP rendezvous, and rank 0's line carries n_gpus 2 and the max over
    ranks of the timed region (rank r sleeps (r + 1) * 10 ms per dry-run step)."""
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_PORT")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "4", "--warmup", "1",
                        "--dry-run"], env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["dry_run"] is True
    assert res["config"]["clips_per_gpu"] == 8 and res["config"]["global_clips"] == 16
    assert res["rendezvous"].startswith("tcp 127.0.0.1")
    assert len(res["rank_ms"]) == 2 and res["rank_ms"][1] >= 4 * 20.0
    assert abs(res["ms_per_step"] - max(res["rank_ms"]) / 4) < 1e-2
    assert abs(res["value"] / (2 * 8 * 30.0 * 4 / (max(res["rank_ms"]) / 1e3)) - 1) < 1e-3


def _launcher(extra_env, *args, timeout=120):
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_PORT", "WMI_TEST_FAIL_RANK", "WMI_TEST_HANG_RANK")}
    env.update(extra_env)
    t0 = time.monotonic()
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run"] + list(args),
                       env=env, capture_output=True, text=True, timeout=timeout)
    return p, time.monotonic() - t0


def test_bench_launcher_fails_when_a_rank_fails():
    """Rank 1 exits with status 3 after the rendezvous while rank 0 hangs
    (as a rank blocked inside RCCL would): the launcher kills rank 0 at once —
    long before its deadline — and exits with rank 1's status, without a
    result line.  Without the hang, rank 0 notices the closed peer itself and
    the launcher still exits non-zero."""
    p, el = _launcher({"WMI_TEST_FAIL_RANK": "1", "WMI_TEST_HANG_RANK": "0"}, "--steps", "2", "--warmup", "1")
    assert p.returncode == 3, p.stderr[-2000:]
    assert "rank 1 exited with status 3" in p.stderr
    assert "WMI_TEST_FAIL_RANK" in p.stderr  # the rank got past the rendezvous before failing
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert el < 60
    p, _ = _launcher({"WMI_TEST_FAIL_RANK": "1"}, "--steps", "2", "--warmup", "1")
    assert p.returncode != 0 and "stopping the other ranks" in p.stderr


def test_bench_launcher_deadline_kills_a_hung_rank():
    """Rank 1 hangs after the rendezvous: at the deadline the launcher kills
    every rank and exits non-zero (124) instead of polling forever."""
    p, el = _launcher({"WMI_TEST_HANG_RANK": "1"}, "--steps", "2", "--warmup", "1", "--launch-deadline", "8")
    assert p.returncode == 124, p.stderr[-2000:]
    assert "deadline of 8 s passed" in p.stderr
    assert 8 <= el < 60


def test_rendezvous_skips_a_busy_hub_port():
    """The first hub port is held by another listener that never answers the
    handshake: rank 0 binds the next candidate and rank 1 finds it there."""
    import threading

    import dist
    base = _free_port()
    ports = dist.hub_ports(base)
    squatter = socket.socket()
    squatter.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
    try:
        squatter.bind(("127.0.0.1", ports[0]))
    except OSError:
        import pytest
        pytest.skip("candidate port taken")
    squatter.listen(4)
    old = os.environ.get("MASTER_PORT")
    os.environ["MASTER_PORT"] = str(base)
    try:
        res = {}

        def hub():
            g = dist.Group(0, 2, "127.0.0.1", timeout=30)
            res["gather"] = g.all_gather("hub")
            g.close()

        t = threading.Thread(target=hub)
        t.start()
        peer = dist.Group(1, 2, "127.0.0.1", timeout=30)
        assert peer.all_gather("peer") == ["hub", "peer"]
        peer.close()
        t.join(30)
        assert res["gather"] == ["hub", "peer"]
    finally:
        squatter.close()
        if old is None:
            del os.environ["MASTER_PORT"]
        else:
            os.environ["MASTER_PORT"] = old


def test_rendezvous_messages_are_data_only():
    """The TCP star carries JSON (bytes hex-tagged), never pickles."""
    import dist
    obj = [b"\x00\x01uid", 1.5, None, [1, 2, 3], "s"]
    assert dist._dec(dist._enc(obj)) == obj
    import pytest
    with pytest.raises(TypeError):
        dist._enc(object())
    with pytest.raises(ValueError):
        dist._dec(b'{"b": "00", "x": 1}')


def test_rendezvous_rejects_bad_ranks():
    """Rank 0 drops peers announcing an out-of-range or duplicate rank."""
    import struct
    import threading

    import dist
    port = _free_port()
    res = {}

    def hub():
        g = dist.Group(0, 2, "127.0.0.1", port, timeout=30)
        res["gather"] = g.all_gather("hub")
        g.close()

    t = threading.Thread(target=hub)
    t.start()
    import time
    for _ in range(100):  # the hub is listening once a connection succeeds
        try:
            rogue = socket.create_connection(("127.0.0.1", port), timeout=5)
            break
        except OSError:
            time.sleep(0.05)
    dist._send(rogue, struct.pack("<i", 7))  # world is 2: rank 7 is refused
    rogue.settimeout(5)
    assert rogue.recv(1) == b""  # closed by the hub
    rogue.close()
    peer = dist.Group(1, 2, "127.0.0.1", port, timeout=30)
    assert peer.all_gather("peer") == ["hub", "peer"]
    peer.close()
    t.join(30)
    assert res["gather"] == ["hub", "peer"]


def test_rendezvous_survives_a_silent_connection():
    """A connection that sends nothing holds rank 0 for its per-connection
    handshake timeout; the real peer connecting meanwhile waits longer than
    that for its ack (dist._HS_PEER > dist._HS_HUB), so it is acked and
    confirmed once rank 0 gives up on the silent one."""
    import threading
    import time

    import dist
    port = _free_port()
    res = {}
    old = dist._HS_HUB
    dist._HS_HUB = 2.0  # (keeps the test short; the ordering is what matters)
    try:
        def hub():
            g = dist.Group(0, 2, "127.0.0.1", port, timeout=30)
            res["gather"] = g.all_gather("hub")
            g.close()

        t = threading.Thread(target=hub)
        t.start()
        for _ in range(100):
            try:
                silent = socket.create_connection(("127.0.0.1", port), timeout=5)
                break
            except OSError:
                time.sleep(0.05)
        peer = dist.Group(1, 2, "127.0.0.1", port, timeout=30)
        assert peer.all_gather("peer") == ["hub", "peer"]
        peer.close()
        silent.close()
        t.join(30)
        assert res["gather"] == ["hub", "peer"]
    finally:
        dist._HS_HUB = old


def test_rendezvous_duplicate_rank_keeps_the_live_peer():
    """A second process announcing a rank that already joined (with the full
    handshake) is refused while the first one's socket is open; the first
    peer stays in the group.  A rank whose first connection died
    after its handshake is replaced by its reconnect."""
    import struct
    import threading
    import time

    import dist

    def connect(port):
        for _ in range(100):
            try:
                return socket.create_connection(("127.0.0.1", port), timeout=5)
            except OSError:
                time.sleep(0.05)
        raise OSError("hub not listening")

    def handshake(s, port, rank, world):
        hello = dist._MAGIC + struct.pack("<ii", world, port)
        dist._send(s, hello + struct.pack("<i", rank))
        s.settimeout(5)
        assert dist._recv(s) == hello
        dist._send(s, dist._CONFIRM)

    # (1) live duplicate: refused, the first rank 1 stays
    port = _free_port()
    res = {}

    def hub3():
        g = dist.Group(0, 3, "127.0.0.1", port, timeout=30)
        res["gather"] = g.all_gather("hub")
        g.close()

    t = threading.Thread(target=hub3)
    t.start()
    first = {}
    t1 = threading.Thread(target=lambda: first.setdefault("g", dist.Group(1, 3, "127.0.0.1", port, timeout=30)))
    t1.start()
    t1.join(30)
    imp = connect(port)
    handshake(imp, port, 1, 3)
    assert imp.recv(1) == b""  # closed by the hub: rank 1 is taken by a live peer
    imp.close()
    out = {}
    t2 = threading.Thread(target=lambda: out.setdefault("r2", dist.Group(2, 3, "127.0.0.1", port, timeout=30)
                                                         .all_gather("two")))
    t2.start()
    assert first["g"].all_gather("one") == ["hub", "one", "two"]
    t2.join(30)
    t.join(30)
    assert res["gather"] == ["hub", "one", "two"] and out["r2"] == ["hub", "one", "two"]
    first["g"].close()

    # (2) dead first connection: the reconnect replaces it
    port = _free_port()
    res.clear()

    def hub2():
        g = dist.Group(0, 3, "127.0.0.1", port, timeout=30)
        res["gather"] = g.all_gather("hub")
        g.close()

    t = threading.Thread(target=hub2)
    t.start()
    dead = connect(port)
    handshake(dead, port, 1, 3)
    dead.close()
    time.sleep(0.2)
    again = {}
    t1 = threading.Thread(target=lambda: again.setdefault("g", dist.Group(1, 3, "127.0.0.1", port, timeout=30)))
    t1.start()
    t1.join(30)
    out.clear()
    t2 = threading.Thread(target=lambda: out.setdefault("r2", dist.Group(2, 3, "127.0.0.1", port, timeout=30)
                                                         .all_gather("two")))
    t2.start()
    assert again["g"].all_gather("one") == ["hub", "one", "two"]
    t2.join(30)
    t.join(30)
    assert res["gather"] == ["hub", "one", "two"]
    again["g"].close()
