"""Prometheus metrics with the reference names plus the
MI355X training metrics.

Reference names: ``pytorch_operator_is_leader`` (server.go:58-61),
``pytorch_operator_jobs_created_total`` (job.go:28-31),
``pytorch_operator_jobs_deleted_total`` (controller.go:67-70),
``pytorch_operator_jobs_{successful,failed,restarted}_total``
(status.go:48-59).  Each controller instance owns a registry so tests can
run several side by side.
"""
from __future__ import annotations

from prometheus_client import CollectorRegistry, Counter, Gauge, Histogram, generate_latest


class OperatorMetrics:
    def __init__(self, registry: CollectorRegistry | None = None):
        self.registry = registry or CollectorRegistry()
        r = self.registry
        self.is_leader = Gauge("pytorch_operator_is_leader", "Is this client the leader of this pytorch-operator "
                                                             "client set?", registry=r)
        self.jobs_created = Counter("pytorch_operator_jobs_created", "Counts number of PyTorch jobs created",
                                    registry=r)
        self.jobs_deleted = Counter("pytorch_operator_jobs_deleted", "Counts number of PyTorch jobs deleted",
                                    registry=r)
        self.jobs_successful = Counter("pytorch_operator_jobs_successful",
                                       "Counts number of PyTorch jobs successful", registry=r)
        self.jobs_failed = Counter("pytorch_operator_jobs_failed", "Counts number of PyTorch jobs failed",
                                   registry=r)
        self.jobs_restarted = Counter("pytorch_operator_jobs_restarted",
                                      "Counts number of PyTorch jobs restarted", registry=r)
        self.sync_seconds = Histogram("pytorch_operator_sync_duration_seconds", "PyTorchJob sync latency",
                                      registry=r, buckets=(.0005, .001, .0025, .005, .01, .025, .05, .1, .25, 1))
        # MI355X training metrics (fed by the node agent / trainer reports)
        self.samples_per_second = Gauge("pytorchjob_samples_per_second", "Training throughput",
                                        ["job", "replica"], registry=r)
        self.step_seconds = Gauge("pytorchjob_step_seconds", "Training step time", ["job", "replica"], registry=r)
        self.allreduce_seconds = Gauge("pytorchjob_allreduce_seconds", "Gradient all-reduce time per step",
                                       ["job", "replica"], registry=r)
        self.submit_to_first_step = Gauge("pytorchjob_submit_to_first_step_seconds",
                                          "creationTimestamp -> first optimizer step on rank 0", ["job"],
                                          registry=r)
        self.gpu_hbm_used = Gauge("pytorchjob_gpu_hbm_used_bytes", "HBM used per GPU", ["gpu"], registry=r)
        self.gpu_hbm_total = Gauge("pytorchjob_gpu_hbm_total_bytes", "HBM total per GPU", ["gpu"], registry=r)

    def exposition(self) -> bytes:
        return generate_latest(self.registry)


def serve_metrics(metrics: OperatorMetrics, port: int, host: str = "0.0.0.0"):
    """Serve ``/metrics`` on ``--monitoring-port`` (main.go:31-40)."""
    from prometheus_client import start_http_server

    return start_http_server(port, addr=host, registry=metrics.registry)
