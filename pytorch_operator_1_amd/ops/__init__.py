"""gfx950 HIP operators (see ``csrc/kernels``) and their autograd wrappers."""
from .nn import conv2d_bias_relu_maxpool, cross_entropy, linear, log_softmax  # noqa: F401
from .optim import FusedSGD, SgdTable  # noqa: F401
