"""Wire-level constants of the ``kubeflow.org/v1`` PyTorchJob API.

Every value here is part of the external contract and must match the
reference byte for byte:

* group/version/kind/plural — ``pkg/apis/pytorch/v1/register.go:31-74``
* default port / container / restart policy — ``pkg/apis/pytorch/v1/constants.go:20-34``
* common condition types, clean-pod and restart policies —
  vendored ``kubeflow/common/job_controller/api/v1/types.go:101-156``
* label keys — vendored ``jobcontroller.go:196-222``,
  ``pkg/controller.v1/pytorch/controller.go:55-58``
* reasons — ``status.go:34-45``, ``job.go:24``, ``pod.go:36-45``
"""

GROUP_NAME = "kubeflow.org"
VERSION = "v1"
API_VERSION = f"{GROUP_NAME}/{VERSION}"
KIND = "PyTorchJob"
LIST_KIND = "PyTorchJobList"
PLURAL = "pytorchjobs"
SINGULAR = "pytorchjob"
CRD_NAME = f"{PLURAL}.{GROUP_NAME}"
CONTROLLER_NAME = "pytorch-operator"

ENV_KUBEFLOW_NAMESPACE = "KUBEFLOW_NAMESPACE"
DEFAULT_PORT_NAME = "pytorchjob-port"
DEFAULT_CONTAINER_NAME = "pytorch"
DEFAULT_PORT = 23456
DEFAULT_RESTART_POLICY = "OnFailure"

# replica types
REPLICA_MASTER = "Master"
REPLICA_WORKER = "Worker"
REPLICA_TYPES = (REPLICA_MASTER, REPLICA_WORKER)

# job condition types
JOB_CREATED = "Created"
JOB_RUNNING = "Running"
JOB_RESTARTING = "Restarting"
JOB_SUCCEEDED = "Succeeded"
JOB_FAILED = "Failed"
CONDITION_TYPES = (JOB_CREATED, JOB_RUNNING, JOB_RESTARTING, JOB_SUCCEEDED, JOB_FAILED)

# clean pod policy
CLEAN_POD_POLICY_UNDEFINED = ""
CLEAN_POD_POLICY_ALL = "All"
CLEAN_POD_POLICY_RUNNING = "Running"
CLEAN_POD_POLICY_NONE = "None"

# restart policy
RESTART_POLICY_ALWAYS = "Always"
RESTART_POLICY_ON_FAILURE = "OnFailure"
RESTART_POLICY_NEVER = "Never"
RESTART_POLICY_EXIT_CODE = "ExitCode"
RESTART_POLICIES = (RESTART_POLICY_ALWAYS, RESTART_POLICY_ON_FAILURE, RESTART_POLICY_NEVER, RESTART_POLICY_EXIT_CODE)

# labels
LABEL_GROUP_NAME = "group-name"
LABEL_JOB_NAME = "job-name"
LABEL_PYTORCH_JOB_NAME = "pytorch-job-name"
LABEL_CONTROLLER_NAME = "controller-name"
LABEL_REPLICA_TYPE = "pytorch-replica-type"
LABEL_REPLICA_INDEX = "pytorch-replica-index"
LABEL_JOB_ROLE = "job-role"
ANNOTATION_GANG_GROUP = "scheduling.k8s.io/group-name"

# reasons
REASON_CREATED = "PyTorchJobCreated"
REASON_RUNNING = "PyTorchJobRunning"
REASON_SUCCEEDED = "PyTorchJobSucceeded"
REASON_FAILED = "PyTorchJobFailed"
REASON_RESTARTING = "PyTorchJobRestarting"
REASON_INVALID_SPEC = "InvalidPyTorchJobSpec"
REASON_POD_TEMPLATE_RESTART_POLICY = "SettedPodTemplateRestartPolicy"
REASON_EXITED_WITH_CODE = "ExitedWithCode"
REASON_POD_TEMPLATE_SCHEDULER_NAME = "SettedPodTemplateSchedulerName"

# MI355X resource name (replaces nvidia.com/gpu in the reference YAML)
GPU_RESOURCE = "amd.com/gpu"
LEGACY_GPU_RESOURCES = ("nvidia.com/gpu",)
HBM_PER_GPU_BYTES = 288 * 1000 ** 3  # MI355X: 288 GB HBM3E
# per-replica HBM request (bytes per GPU, k8s quantity), checked against the GPU's HBM
HBM_RESOURCE = "amd.com/hbm"

# controller tunables (reference values)
EXPECTATIONS_TIMEOUT_S = 5 * 60
JOB_RESYNC_PERIOD_S = 30
RECONCILER_SYNC_LOOP_PERIOD_S = 15
LEADER_LEASE_S, LEADER_RENEW_S, LEADER_RETRY_S = 15, 5, 3
