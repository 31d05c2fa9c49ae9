"""Native node agent protocol tests (kubelet restart semantics, exit codes,
gang GPU allocation, TCP probe).  They drive the ASan+UBSan build of the
agent (host-only sanitizers) unless ``PTO_NODE_AGENT_BIN`` names another
binary, so memory errors in the C++ supervisor fail the suite."""
import os
import socket
import sys
import time

import pytest

from pytorch_operator_1_amd.node import native


@pytest.fixture(scope="module")
def agent():
    binary = os.environ.get("PTO_NODE_AGENT_BIN") or native.build(sanitize=True)
    a = native.AgentClient(gpus=4, hbm_per_gpu=288e9, backoff_base=0.05, backoff_max=0.2, binary=binary)
    yield a
    a.close()
    if a._proc is not None:
        assert a._proc.returncode == 0, "sanitized agent exited non-zero (sanitizer report on stderr)"


def wait_state(agent, pid, pred, timeout=10.0):
    end = time.time() + timeout
    while time.time() < end:
        st = agent.status(pid)[pid]
        if pred(st):
            return st
        time.sleep(0.02)
    raise AssertionError(agent.status(pid)[pid])


def test_ping(agent):
    r = agent.call("ping")
    assert r["ok"] and r["gpus"] == 4


def test_exit_codes_and_completed(agent, tmp_path):
    log = tmp_path / "a.log"
    agent.spawn("ok", [sys.executable, "-c", "print('hello')"], log=str(log))
    st = wait_state(agent, "ok", lambda s: s["state"] == "terminated")
    assert st["exit_code"] == 0 and st["reason"] == "Completed"
    assert "hello" in log.read_text()
    agent.spawn("bad", [sys.executable, "-c", "import sys; sys.exit(3)"])
    st = wait_state(agent, "bad", lambda s: s["state"] == "terminated")
    assert st["exit_code"] == 3 and st["reason"] == "Error"


def test_exec_failure_is_reported(agent):
    agent.spawn("noexec", ["/nonexistent/binary"])
    st = wait_state(agent, "noexec", lambda s: s["state"] == "terminated" or s["reason"] == "StartError")
    assert st["reason"] in ("StartError", "Error")


def test_onfailure_restarts_with_backoff(agent, tmp_path):
    marker = tmp_path / "count"
    code = (f"import os,sys; p={str(marker)!r}; n=int(open(p).read()) if os.path.exists(p) else 0; "
            f"open(p,'w').write(str(n+1)); sys.exit(0 if n>=2 else 1)")
    agent.spawn("flaky", [sys.executable, "-c", code], restart_policy="OnFailure")
    st = wait_state(agent, "flaky", lambda s: s["state"] == "terminated")
    assert st["exit_code"] == 0 and st["restart_count"] == 2 and st["last_exit_code"] == 1


def test_signal_exit_code_and_kill(agent):
    agent.spawn("sleeper", [sys.executable, "-c", "import time; time.sleep(60)"])
    wait_state(agent, "sleeper", lambda s: s["state"] == "running")
    agent.kill("sleeper", signal=9)
    st = wait_state(agent, "sleeper", lambda s: s["state"] == "terminated")
    assert st["exit_code"] == 137 and st["signal"] == 9 and st["reason"] == "Killed"
    assert agent.remove("sleeper")["ok"]
    assert "sleeper" not in agent.status()


def test_restartable_kill_is_fault_injection(agent):
    agent.spawn("victim", [sys.executable, "-c", "import time; time.sleep(60)"], restart_policy="OnFailure")
    wait_state(agent, "victim", lambda s: s["state"] == "running")
    agent.kill("victim", signal=9, restartable=True)
    st = wait_state(agent, "victim", lambda s: s["restart_count"] == 1 and s["state"] == "running")
    assert st["last_exit_code"] == 137
    agent.kill("victim", signal=9)
    wait_state(agent, "victim", lambda s: s["state"] == "terminated")


def test_gang_alloc_all_or_nothing(agent):
    r = agent.alloc([{"owner": "j1-master-0", "count": 1, "hbm": 100e9}, {"owner": "j1-worker-0", "count": 2}])
    assert r["ok"] and len(r["assigned"]["j1-worker-0"]) == 2
    r2 = agent.alloc([{"owner": "j2-master-0", "count": 1}, {"owner": "j2-worker-0", "count": 1}])
    assert not r2["ok"] and r2.get("unschedulable")
    owners = [g["owner"] for g in agent.gpus()["gpus"]]
    assert "j2-master-0" not in owners  # nothing partially allocated
    again = agent.alloc([{"owner": "j1-master-0", "count": 1}])  # idempotent
    assert again["assigned"]["j1-master-0"] == r["assigned"]["j1-master-0"]
    too_big = agent.alloc([{"owner": "big", "count": 1, "hbm": 300e9}])
    assert not too_big["ok"] and "HBM" in too_big["error"]
    assert agent.free("j1-master-0")["freed"] == 1
    assert agent.free("j1-worker-0")["freed"] == 2


def test_tcp_probe(agent):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    s.listen(1)
    port = s.getsockname()[1]
    assert agent.probe("127.0.0.1", port)
    s.close()
    assert not agent.probe("127.0.0.1", port, timeout=0.2)
