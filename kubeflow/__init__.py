# namespace shim so `from kubeflow.pytorchjob import PyTorchJobClient` works
