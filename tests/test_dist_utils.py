"""Backend resolution of the trainer's --backend flag (reference choices
gloo|nccl|mpi, examples/mnist/mnist.py:99-102, plus rccl)."""
import pytest
import torch.distributed as dist

from pytorch_operator_1_amd.utils.dist import resolve_backend


def test_aliases():
    assert resolve_backend("rccl", True) == "nccl"
    assert resolve_backend("NCCL", True) == "nccl"
    assert resolve_backend("gloo", True) == "gloo"
    assert resolve_backend(None, True) == "nccl"
    assert resolve_backend(None, False) == "gloo"
    with pytest.raises(ValueError):
        resolve_backend("ucc", False)


def test_mpi_falls_back_without_mpi_support(capsys):
    if dist.is_mpi_available():
        assert resolve_backend("mpi", False) == "mpi"
        return
    assert resolve_backend("mpi", True) == "nccl"
    assert resolve_backend("mpi", False) == "gloo"
    assert "no MPI support" in capsys.readouterr().err
