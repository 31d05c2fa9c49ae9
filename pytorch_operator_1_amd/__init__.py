"""MI355X-native PyTorchJob operator + training runtime (capabilities of kubeflow pytorch-operator v1)."""
__version__ = "0.1.0"
