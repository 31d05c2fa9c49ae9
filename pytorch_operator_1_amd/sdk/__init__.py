"""PyTorchJob Python SDK (API-compatible with ``kubeflow-pytorchjob``)."""
from .client import PyTorchJobClient  # noqa: F401
from .models import *  # noqa: F401,F403
