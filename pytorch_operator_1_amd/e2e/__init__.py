"""End-to-end drivers mirroring the reference's ``test/e2e/v1`` programs.

``python -m pytorch_operator_1_amd.e2e.defaults`` and
``python -m pytorch_operator_1_amd.e2e.cleanpolicy_all`` run N concurrent
PyTorchJobs against a live API server (``--server``) or an in-process
:class:`~pytorch_operator_1_amd.cluster.LocalCluster` (``--local``), and
exit non-zero unless every job behaves as specified.
"""
