"""Tracing helpers: torch.profiler Chrome trace per rank from the trainer
CLI, and the HIP-event step timer's disabled (CPU) path."""
import json
import os

from pytorch_operator_1_amd.utils.profiling import StepTimer, torch_trace


def test_step_timer_disabled_on_cpu():
    t = StepTimer("cpu")
    with t.phase("forward"):
        pass
    assert t.summary() == {}


def test_torch_trace_written(tmp_path):
    import torch

    with torch_trace(str(tmp_path), rank=3, active_steps=2) as step:
        for _ in range(5):
            torch.ones(8).sum()
            step()
    p = tmp_path / "trace_rank3.json"
    assert p.exists()
    assert "traceEvents" in json.loads(p.read_text())


def test_mnist_cli_profile_flag(tmp_path):
    from pytorch_operator_1_amd.train import mnist

    os.environ["PTO_NO_GPU"] = "1"
    try:
        assert mnist.main(["--no-cuda", "--max-steps", "15", "--train-size", "1280", "--no-test",
                           "--profile", str(tmp_path)]) == 0
    finally:
        os.environ.pop("PTO_NO_GPU")
    assert (tmp_path / "trace_rank0.json").exists()
