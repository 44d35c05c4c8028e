"""Failure detection / recovery (SURVEY §4.4 "chief restart from checkpoint (kill -9 the chief, then relaunch)",
§5 heartbeats + fault injection)."""
import os
import subprocess
import sys
import time

import pytest

from distributed_tensorflow_amd.parallel import fault
from distributed_tensorflow_amd.parallel.kv import KVClient, KVServer

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(**kw):
    e = dict(os.environ)
    e["PYTHONPATH"] = ROOT + (os.pathsep + e["PYTHONPATH"] if e.get("PYTHONPATH") else "")
    e.update(kw)
    return e


def test_fault_spec_parsing():
    f = fault.FaultInjector("kill@step=5@role=master0", role="worker0")
    assert f.action == "kill" and f.trigger == "step" and f.at == 5 and not f.armed
    g = fault.FaultInjector("raise@step=3", role="x")
    g.on_step(2)
    with pytest.raises(RuntimeError):
        g.on_step(3)
    g.on_step(4)  # fires once
    with pytest.raises(ValueError):
        fault.FaultInjector("explode@step=1")


def test_retry_and_heartbeat_monitor():
    calls = []

    def flaky():
        calls.append(1)
        if len(calls) < 3:
            raise ConnectionError("transient")
        return 7
    assert fault.retry(flaky, retries=3, backoff_s=0.01) == 7 and len(calls) == 3
    srv = KVServer("127.0.0.1", 0)
    try:
        kv = KVClient("127.0.0.1", srv.port)
        hb = fault.Heartbeat(kv, "worker0", interval=0.1).start()
        mon = fault.HeartbeatMonitor(kv, ["worker0", "ps0"])
        time.sleep(0.35)
        assert mon.dead(timeout=1.0) == ["ps0"]  # never beat
        hb.stop()
        assert hb.beats >= 3
        assert "worker0" in mon.dead(timeout=0.5, now=time.time() + 1.0)  # stale once it stopped
        kv.close()
    finally:
        srv.stop()


def test_heartbeat_detects_killed_process():
    srv = KVServer("127.0.0.1", 0)
    try:
        code = ("import sys,time; sys.path.insert(0, %r)\n"
                "from distributed_tensorflow_amd.parallel.kv import KVClient\n"
                "from distributed_tensorflow_amd.parallel.fault import Heartbeat\n"
                "hb = Heartbeat(KVClient('127.0.0.1', %d), 'worker1', interval=0.1).start()\n"
                "time.sleep(60)\n") % (ROOT, srv.port)
        p = subprocess.Popen([sys.executable, "-c", code], env=_env())
        kv = KVClient("127.0.0.1", srv.port)
        mon = fault.HeartbeatMonitor(kv, ["worker1"])
        t0 = time.time()
        while mon.last_seen("worker1") is None and time.time() - t0 < 60:
            time.sleep(0.1)
        assert mon.dead(timeout=1.0) == []
        p.kill()
        p.wait()
        time.sleep(1.5)
        assert mon.dead(timeout=1.0) == ["worker1"]
        kv.close()
    finally:
        srv.stop()


@pytest.mark.slow
def test_chief_kill9_restart_restores_from_checkpoint(tmp_path):
    """ps + worker + master; the master is SIGKILLed right after its first checkpoint, the supervising
    launcher restarts it, it restores from the checkpoint, training finishes, the PS auto-stops, the
    chief exports."""
    cmd = [sys.executable, "-m", "distributed_tensorflow_amd.cli.launch", "--ps", "1", "--workers", "1",
           "--chief", "1", "--max_restarts", "1", "--timeout", "240", "--", sys.executable, "-m",
           "distributed_tensorflow_amd.cli.train", "--seed=0", "--max_epochs=40", "--optimizer=sgd",
           "--save_model_secs=1"]
    r = subprocess.run(cmd, cwd=tmp_path, env=_env(DTF_FAULT="kill@ckpt=1@role=master0"), capture_output=True,
                       text=True, timeout=300)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "[fault] injecting kill at checkpoint 1 (master0)" in out
    assert "master0 exited with -9; restart 1/1" in out
    assert "Restored from" in out
    assert "PS exits after all workers done" in out
    assert "Exported SavedModel" in out
    assert os.path.isdir(tmp_path / "saved_model" / "1")
