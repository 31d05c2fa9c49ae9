"""Drop-in import path of the reference SDK (``kubeflow.pytorchjob``),
backed by :mod:`pytorch_operator_1_amd.sdk`."""
from pytorch_operator_1_amd.sdk import *  # noqa: F401,F403
from pytorch_operator_1_amd.sdk import PyTorchJobClient  # noqa: F401
from pytorch_operator_1_amd.sdk import constants, utils  # noqa: F401
