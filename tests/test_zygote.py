"""Warm starts: the node agent's zygote (``node/zygote.py``) forks
containers from a pre-imported interpreter.  The container must behave like
a fork/exec'ed one: argv, env (only the pod's), cwd, log capture, exit codes,
signals -> 128+n, restart policy, process-group kill; non-Python argv takes
the exec path.  Runs the ASan/UBSan agent build like test_node_agent.py."""
import json
import os
import sys
import time

import pytest

from pytorch_operator_1_amd.node import native

SCRIPT = r'''
import json, os, sys, time
out = {"argv": sys.argv, "env": dict(os.environ), "cwd": os.getcwd(), "pid": os.getpid(),
       "pgid": os.getpgid(0), "ppid": os.getppid(), "torch_loaded": "torch" in sys.modules,
       "main": __name__}
print("STDOUT-LINE", flush=False)
print("STDERR-LINE", file=sys.stderr)
with open(os.environ["OUT"], "w") as f:
    json.dump(out, f)
mode = sys.argv[1] if len(sys.argv) > 1 else ""
if mode == "sleep":
    time.sleep(60)
if mode == "raise":
    raise ValueError("boom")
sys.exit(int(sys.argv[2]) if len(sys.argv) > 2 else 0)
'''


@pytest.fixture(scope="module")
def agent():
    binary = os.environ.get("PTO_NODE_AGENT_BIN") or native.build(sanitize=True)
    a = native.AgentClient(gpus=2, backoff_base=0.05, backoff_max=0.2, binary=binary, zygote=True)
    assert a.wait_warm(120), a.ping()
    yield a
    a.close()
    if a._proc is not None:
        assert a._proc.returncode == 0, "sanitized agent exited non-zero (sanitizer report on stderr)"


def wait_state(agent, pid, pred, timeout=30.0):
    end = time.time() + timeout
    while time.time() < end:
        st = agent.status(pid)[pid]
        if pred(st):
            return st
        time.sleep(0.02)
    raise AssertionError(agent.status(pid)[pid])


def _script(tmp_path):
    p = tmp_path / "probe.py"
    p.write_text(SCRIPT)
    return str(p)


def test_zygote_container_argv_env_cwd_log_exit(agent, tmp_path):
    out = tmp_path / "out.json"
    log = tmp_path / "c.log"
    cwd = tmp_path / "work"
    cwd.mkdir()
    env = {"OUT": str(out), "HIP_VISIBLE_DEVICES": "1", "RANK": "0", "PATH": os.environ.get("PATH", "")}
    agent.spawn("z/exit", [sys.executable, _script(tmp_path), "exit", "3"], env=env, cwd=str(cwd), log=str(log))
    st = wait_state(agent, "z/exit", lambda s: s["state"] == "terminated")
    assert st["launcher"] == "zygote"
    assert st["exit_code"] == 3 and st["reason"] == "Error"
    info = json.loads(out.read_text())
    assert info["argv"][1:] == ["exit", "3"] and info["main"] == "__main__"
    assert info["env"]["HIP_VISIBLE_DEVICES"] == "1" and "PYTHONPATH" not in info["env"]
    # + the store backend a fork can run, and the launcher's startup timestamps
    assert set(info["env"]) <= set(env) | {"PWD", "USE_LIBUV", "PTO_ZYGOTE_T"}
    assert info["env"]["USE_LIBUV"] == "0"
    assert info["cwd"] == str(cwd)
    assert info["torch_loaded"]  # warm: torch came from the zygote's imports
    assert info["pgid"] == info["pid"]  # own session / process group
    text = log.read_text()
    assert "STDOUT-LINE" in text and "STDERR-LINE" in text
    assert agent.ping()["zygote"]["spawned"] >= 1


def test_zygote_module_form_and_uncaught_exception(agent, tmp_path):
    out = tmp_path / "out.json"
    log = tmp_path / "m.log"
    pkg = tmp_path / "zmod"
    pkg.mkdir()
    (pkg / "__init__.py").write_text("")
    (pkg / "probe.py").write_text(SCRIPT)
    env = {"OUT": str(out), "PATH": os.environ.get("PATH", "")}
    agent.spawn("z/mod", [sys.executable, "-m", "zmod.probe", "raise"], env=env, cwd=str(tmp_path), log=str(log))
    st = wait_state(agent, "z/mod", lambda s: s["state"] == "terminated")
    assert st["launcher"] == "zygote" and st["exit_code"] == 1
    assert "ValueError: boom" in log.read_text()
    assert json.loads(out.read_text())["argv"][0].endswith("probe.py")


def test_zygote_signal_exit_code_and_restart(agent, tmp_path):
    out = tmp_path / "out.json"
    env = {"OUT": str(out), "PATH": os.environ.get("PATH", "")}
    agent.spawn("z/sleep", [sys.executable, _script(tmp_path), "sleep"], env=env, log=str(tmp_path / "s.log"),
                restart_policy="OnFailure")
    st = wait_state(agent, "z/sleep", lambda s: s["state"] == "running" and out.exists())
    pid1 = st["pid"]
    assert st["launcher"] == "zygote"
    agent.kill("z/sleep", signal=9, restartable=True)  # fault injection: SIGKILL -> 137, retryable
    st = wait_state(agent, "z/sleep", lambda s: s["restart_count"] >= 1 and s["state"] == "running")
    assert st["last_exit_code"] == 137 and st["pid"] != pid1 and st["launcher"] == "zygote"
    agent.kill("z/sleep", signal=15, grace=2.0)
    st = wait_state(agent, "z/sleep", lambda s: s["state"] == "terminated")
    assert st["exit_code"] == 143 and st["reason"] == "Killed"


def test_non_python_argv_takes_exec_path(agent, tmp_path):
    agent.spawn("z/sh", ["/bin/sh", "-c", "exit 5"], env={"PATH": "/usr/bin:/bin"})
    st = wait_state(agent, "z/sh", lambda s: s["state"] == "terminated")
    assert st["launcher"] == "exec" and st["exit_code"] == 5
    # interpreter flags the zygote cannot honour -> exec
    agent.spawn("z/X", [sys.executable, "-X", "utf8", "-c", "raise SystemExit(4)"], env={})
    st = wait_state(agent, "z/X", lambda s: s["state"] == "terminated")
    assert st["launcher"] == "exec" and st["exit_code"] == 4


def test_eligibility_rules():
    from pytorch_operator_1_amd.node.zygote import eligible

    py = sys.executable
    assert eligible([py, "-m", "pkg.mod", "--x"], py)
    assert eligible([py, "-u", "train.py"], py)
    assert not eligible([py, "-c", "print(1)"], py)
    assert not eligible([py, "-m"], py)
    assert not eligible(["/bin/sh", "x.py"], py)


def test_exec_only_container_runs_in_a_warm_spare(agent, tmp_path):
    """A container that must not be forked from the zygote (launcher "exec":
    the rendezvous store host of a multi-rank job) runs in the agent's warm
    SPARE interpreter -- an exec'ed process that already did the zygote's
    imports and becomes the container itself -- and a new spare warms up for
    the next one.  Same container contract as a forked one."""
    end = time.time() + 120
    while not agent.ping()["zygote"].get("spare_ready") and time.time() < end:
        time.sleep(0.1)
    assert agent.ping()["zygote"]["spare_ready"]
    used0 = agent.ping()["zygote"]["spares_used"]
    out = tmp_path / "out.json"
    log = tmp_path / "s.log"
    env = {"OUT": str(out), "RANK": "0", "WORLD_SIZE": "2", "PATH": os.environ.get("PATH", "")}
    agent.spawn("z/spare", [sys.executable, _script(tmp_path), "exit", "5"], env=env, log=str(log), launcher="exec")
    st = wait_state(agent, "z/spare", lambda s: s["state"] == "terminated")
    assert st["launcher"] == "spare" and st["exit_code"] == 5
    info = json.loads(out.read_text())
    assert info["argv"][1:] == ["exit", "5"] and info["main"] == "__main__"
    assert info["torch_loaded"]  # warm: imported before the request came
    assert info["pgid"] == info["pid"] and info["env"]["WORLD_SIZE"] == "2"
    text = log.read_text()
    assert "STDOUT-LINE" in text and "STDERR-LINE" in text
    z = agent.ping()["zygote"]
    assert z["spares_used"] == used0 + 1
    end = time.time() + 120  # the replacement warms up
    while not agent.ping()["zygote"].get("spare_ready") and time.time() < end:
        time.sleep(0.1)
    assert agent.ping()["zygote"]["spare_ready"]
    # a killed spare container is reaped like any other
    agent.spawn("z/spare2", [sys.executable, _script(tmp_path), "sleep"], env=env, log=str(log), launcher="exec")
    st = wait_state(agent, "z/spare2", lambda s: s["state"] == "running")
    assert st["launcher"] == "spare"
    agent.kill("z/spare2", signal=9)
    st = wait_state(agent, "z/spare2", lambda s: s["state"] == "terminated")
    assert st["exit_code"] == 137
