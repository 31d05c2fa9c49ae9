"""``pto`` — operator daemon, API server, node agent and kubectl-style CLI.

Daemons
  pto operator   the PyTorchJob controller (reference ``cmd/pytorch-operator.v1``:
                 same flags and defaults, ``options.go:54-83``, incl. the
                 ``--resyc-period`` typo kept for manifest compatibility)
  pto apiserver  the Kubernetes-compatible API server
  pto node       the node manager + native agent for this MI355X node
  pto up         all three in one process (single 8xMI355X node)

Client (talks to ``--server`` / ``$PTO_APISERVER``, default 127.0.0.1:8080)
  pto apply -f job.yaml | pto get pytorchjobs|pods|services|events [NAME]
  pto describe NAME | pto logs NAME [--follow] [--all] | pto delete NAME
  pto watch [NAME] | pto kill POD [--signal 9] | pto crd
"""
from __future__ import annotations

import argparse
import json
import logging
import os
import signal
import sys
import threading
import time

from .. import __version__
from ..api import constants as C


# ------------------------------------------------------------- logging ---
class JsonFormatter(logging.Formatter):
    """logrus JSON formatter equivalent with a filename field
    (``main.go:42-58``)."""

    def format(self, record):
        d = {"level": record.levelname.lower(), "msg": record.getMessage(),
             "time": time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime(record.created)),
             "filename": f"{record.filename}:{record.lineno}"}
        for k in ("job", "uid", "replica-type", "pod"):
            if hasattr(record, k.replace("-", "_")):
                d[k] = getattr(record, k.replace("-", "_"))
        if record.exc_info:
            d["error"] = self.formatException(record.exc_info)
        return json.dumps(d)


def setup_logging(json_format: bool, level=logging.INFO):
    h = logging.StreamHandler(sys.stderr)
    h.setFormatter(JsonFormatter() if json_format else logging.Formatter("%(asctime)s %(levelname)s %(message)s"))
    root = logging.getLogger()
    root.handlers[:] = [h]
    root.setLevel(level)


def setup_signal_handler() -> threading.Event:
    """First SIGINT/SIGTERM closes the stop channel, the second exits 1
    (vendored ``util/signals/signal.go:29-43``)."""
    stop = threading.Event()

    def handler(signum, frame):
        if stop.is_set():
            os._exit(1)
        stop.set()

    signal.signal(signal.SIGINT, handler)
    signal.signal(signal.SIGTERM, handler)
    return stop


def version_string() -> str:
    try:
        import torch

        tv, hip = torch.__version__, getattr(torch.version, "hip", None)
    except Exception:
        tv, hip = "n/a", None
    return (f"API Version: {C.API_VERSION}\nVersion: {__version__}\nGit SHA: {_git_sha()}\n"
            f"Python Version: {sys.version.split()[0]}\nOS/Arch: {os.uname().sysname.lower()}/{os.uname().machine}\n"
            f"Torch: {tv}  HIP: {hip}  GPU arch: gfx950 (MI355X)")


def _git_sha():
    try:
        import subprocess

        return subprocess.run(["git", "rev-parse", "--short", "HEAD"], capture_output=True, text=True,
                              cwd=os.path.dirname(os.path.abspath(__file__)), timeout=5).stdout.strip() or "unknown"
    except Exception:
        return "unknown"


# ------------------------------------------------------------- daemons ---
def add_operator_flags(p):
    p.add_argument("--kubeconfig", default="", help="kubeconfig/pto config file (KUBECONFIG env overrides)")
    p.add_argument("--master", default="", help="API server URL (overrides the config file)")
    p.add_argument("--namespace", default=os.environ.get(C.ENV_KUBEFLOW_NAMESPACE, ""),
                   help="namespace to watch ('' = all)")
    p.add_argument("--threadiness", type=int, default=1)
    p.add_argument("--version", action="store_true")
    p.add_argument("--json-log-format", type=lambda s: s.lower() != "false", default=True)
    p.add_argument("--enable-gang-scheduling", action="store_true")
    p.add_argument("--gang-scheduler-name", default="volcano")
    p.add_argument("--monitoring-port", type=int, default=8443)
    p.add_argument("--resyc-period", default="12h", help="informer resync period (sic, reference flag name)")
    p.add_argument("--init-container-image", default="alpine:3.10")
    p.add_argument("--qps", type=float, default=5)
    p.add_argument("--burst", type=int, default=10)
    p.add_argument("--alsologtostderr", action="store_true", help="accepted for manifest compatibility")
    p.add_argument("-v", type=int, default=0, help="accepted for manifest compatibility")
    p.add_argument("--restart-scope", choices=["job", "pod"], default="job",
                   help="ExitCode restarts of a multi-replica job: job = recreate every replica when one fails "
                        "retryably (a DDP world restarts as a whole); pod = only the failed pod (reference)")


def _server_url(args) -> str:
    if getattr(args, "master", ""):
        return args.master
    cfg = os.environ.get("KUBECONFIG") or getattr(args, "kubeconfig", "")
    if cfg and os.path.exists(cfg):
        from ..sdk.client import _load_config

        url, _ = _load_config(cfg, None)
        if url:
            return url
    return getattr(args, "server", None) or os.environ.get("PTO_APISERVER", "http://127.0.0.1:8080")


def cmd_operator(args):
    if args.version:
        print(version_string())
        return 0
    setup_logging(args.json_log_format)
    stop = setup_signal_handler()
    from ..apiserver.client import RestClient
    from ..apiserver.store import ApiError
    from ..controller.leader import LeaderElector
    from ..controller.metrics import OperatorMetrics, serve_metrics
    from ..controller.pytorch import ControllerConfig, PyTorchController

    client = RestClient(_server_url(args))
    try:  # checkCRDExists (server.go:201-213)
        client.list("pytorchjobs")
    except (ApiError, OSError) as e:
        logging.error("CRD %s does not exist or API server unreachable: %s", C.CRD_NAME, e)
        return 1
    metrics = OperatorMetrics()
    serve_metrics(metrics, args.monitoring_port)
    cfg = ControllerConfig(enable_gang_scheduling=args.enable_gang_scheduling,
                           gang_scheduler_name=args.gang_scheduler_name,
                           init_container_image=args.init_container_image, threadiness=args.threadiness,
                           namespace=args.namespace or None, restart_scope=args.restart_scope)
    ctl = PyTorchController(client, cfg, metrics=metrics)

    def lead():
        metrics.is_leader.set(1)
        ctl.run()

    le = LeaderElector(client)
    le.run(lead, block=False)
    stop.wait()
    le.stop()
    ctl.stop()
    return 0


def cmd_apiserver(args):
    setup_logging(False)
    stop = setup_signal_handler()
    from ..api.crd import crd_manifest
    from ..apiserver.server import ApiServer
    from ..apiserver.store import ApiError, Store

    store = Store(wal_path=args.wal)
    try:
        store.create("customresourcedefinitions", crd_manifest())
    except ApiError:
        pass
    srv = ApiServer(store, host=args.host, port=args.port, token=args.token).start_in_thread()
    logging.info("API server listening on %s", srv.url)
    stop.wait()
    srv.stop()
    store.close()
    return 0


def _hbm(args) -> float:
    from ..api.validation import parse_quantity

    return parse_quantity(args.hbm_per_gpu)


def cmd_node(args):
    setup_logging(False)
    stop = setup_signal_handler()
    from ..apiserver.client import RestClient
    from ..node.kubelet import Kubelet

    agent = None
    if args.node_agent_socket:
        from ..node.native import AgentClient

        agent = AgentClient(socket_path=args.node_agent_socket)
    metrics = None
    if args.monitoring_port:
        from ..controller.metrics import OperatorMetrics, serve_metrics

        metrics = OperatorMetrics()
        serve_metrics(metrics, args.monitoring_port)
    kl = Kubelet(RestClient(_server_url(args)), agent=agent, gpus=args.gpus, log_dir=args.log_dir,
                 node_name=args.node_name, hbm_per_gpu=_hbm(args), gpu_visibility=args.gpu_visibility,
                 metrics=metrics)
    kl.start()
    stop.wait()
    kl.stop()
    return 0


def cmd_up(args):
    setup_logging(False)
    stop = setup_signal_handler()
    from ..cluster import LocalCluster
    from ..controller.metrics import serve_metrics

    c = LocalCluster(gpus=args.gpus, port=args.port, wal_path=args.wal, log_dir=args.log_dir,
                     enable_gang_scheduling=args.enable_gang_scheduling, hbm_per_gpu=_hbm(args),
                     gpu_visibility=args.gpu_visibility, restart_scope=args.restart_scope)
    c.start()
    serve_metrics(c.metrics, args.monitoring_port)
    print(f"pto: API server {c.url}  metrics :{args.monitoring_port}/metrics  "
          f"GPUs {c.kubelet.agent.gpus()['count']}", flush=True)
    stop.wait()
    c.stop()
    return 0


# -------------------------------------------------------------- client ---
def _client(args):
    from ..apiserver.client import RestClient

    return RestClient(_server_url(args))


_RES = {"pytorchjob": "pytorchjobs", "pytorchjobs": "pytorchjobs", "pj": "pytorchjobs", "pod": "pods", "pods": "pods",
        "po": "pods", "service": "services", "services": "services", "svc": "services", "event": "events",
        "events": "events", "ev": "events", "node": "nodes", "nodes": "nodes", "podgroups": "podgroups",
        "lease": "leases", "leases": "leases"}


def cmd_apply(args):
    import yaml

    c = _client(args)
    with open(args.filename) if args.filename != "-" else sys.stdin as f:
        docs = [d for d in yaml.safe_load_all(f) if d]
    for d in docs:
        res = {"PyTorchJob": "pytorchjobs", "Pod": "pods", "Service": "services"}.get(d.get("kind"))
        if res is None:
            print(f"skipping unsupported kind {d.get('kind')}")
            continue
        ns = args.namespace or d.get("metadata", {}).get("namespace") or "default"
        try:
            c.create(res, d, ns)
            print(f"{d['kind'].lower()}.{C.GROUP_NAME if res == 'pytorchjobs' else ''}/{d['metadata']['name']} created")
        except Exception as e:
            from ..apiserver.store import ApiError

            if isinstance(e, ApiError) and e.code == 409:
                cur = c.get(res, ns, d["metadata"]["name"])
                d.setdefault("metadata", {})["resourceVersion"] = cur["metadata"]["resourceVersion"]
                c.update(res, d, ns)
                print(f"{d['kind'].lower()}/{d['metadata']['name']} configured")
            else:
                raise
    return 0


def _age(ts):
    from ..api.types import parse_rfc3339

    t = parse_rfc3339(ts) or time.time()
    s = int(time.time() - t)
    return f"{s}s" if s < 120 else (f"{s // 60}m" if s < 7200 else f"{s // 3600}h")


def cmd_get(args):
    c = _client(args)
    res = _RES.get(args.resource, args.resource)
    ns = args.namespace or "default"
    items = [c.get(res, ns, args.name)] if args.name else c.list(res, None if args.all_namespaces else ns)["items"]
    if args.output == "json":
        print(json.dumps(items if not args.name else items[0], indent=2))
        return 0
    if args.output == "yaml":
        import yaml

        print(yaml.safe_dump(items if not args.name else items[0], sort_keys=False))
        return 0
    if res == "pytorchjobs":
        print(f"{'NAME':<32}{'STATE':<14}{'AGE':<8}")
        for j in items:
            cs = j.get("status", {}).get("conditions") or []
            print(f"{j['metadata']['name']:<32}{(cs[-1]['type'] if cs else ''):<14}"
                  f"{_age(j['metadata'].get('creationTimestamp')):<8}")
    elif res == "pods":
        print(f"{'NAME':<36}{'READY':<7}{'STATUS':<12}{'RESTARTS':<10}{'GPUS':<8}{'AGE':<8}")
        for p in items:
            st = p.get("status", {})
            css = st.get("containerStatuses") or []
            ready = sum(1 for x in css if x.get("ready"))
            rs = sum(int(x.get("restartCount", 0)) for x in css)
            gp = (p["metadata"].get("annotations") or {}).get("pto.amd.com/gpus", "")
            print(f"{p['metadata']['name']:<36}{ready}/{len(p['spec'].get('containers', [])):<5}"
                  f"{st.get('phase', ''):<12}{rs:<10}{gp:<8}{_age(p['metadata'].get('creationTimestamp')):<8}")
    elif res == "events":
        print(f"{'TYPE':<9}{'REASON':<32}{'OBJECT':<36}MESSAGE")
        for e in items:
            io = e.get("involvedObject", {})
            print(f"{e.get('type', ''):<9}{e.get('reason', ''):<32}{io.get('kind', '').lower() + '/' + io.get('name', ''):<36}"
                  f"{e.get('message', '')}")
    else:
        print("NAME")
        for o in items:
            print(o["metadata"]["name"])
    return 0


def cmd_describe(args):
    c = _client(args)
    ns = args.namespace or "default"
    j = c.get("pytorchjobs", ns, args.name)
    import yaml

    print(yaml.safe_dump({"Name": j["metadata"]["name"], "Namespace": ns, "Spec": j.get("spec"),
                          "Status": j.get("status")}, sort_keys=False))
    # what each replica process really got (the node manager resolves the
    # master Service name to the node address and virtualises the port)
    pods = [p for p in c.list("pods", ns)["items"]
            if (p["metadata"].get("labels") or {}).get(C.LABEL_JOB_NAME) == args.name]
    if pods:
        print("Replica processes (effective env):")
        for p in sorted(pods, key=lambda p: p["metadata"]["name"]):
            ann = p["metadata"].get("annotations") or {}
            eff = ann.get("pto.amd.com/effective-env")
            print(f"  {p['metadata']['name']}: {eff or '(not started)'}")
    evs = [e for e in c.list("events", ns)["items"] if e.get("involvedObject", {}).get("name") == args.name]
    print("Events:")
    for e in evs:
        print(f"  {e.get('type', ''):<8} {e.get('reason', ''):<28} {e.get('message', '')}")
    return 0


def cmd_logs(args):
    from ..sdk.client import PyTorchJobClient

    cl = PyTorchJobClient(base_url=_server_url(args))
    logs = cl.get_logs(args.name, namespace=args.namespace or "default", master=not args.all, follow=args.follow)
    for pod, text in sorted(logs.items()):
        if len(logs) > 1:
            print(f"==> {pod} <==")
        print(text, end="" if text.endswith("\n") else "\n")
    return 0


def cmd_delete(args):
    c = _client(args)
    res = _RES.get(args.resource, args.resource)
    c.delete(res, args.namespace or "default", args.name)
    print(f"{res}/{args.name} deleted")
    return 0


def cmd_watch(args):
    from ..sdk.watch import watch

    watch(_client(args), name=args.name, namespace=args.namespace or "default", timeout_seconds=args.timeout)
    return 0


def cmd_crd(args):
    import yaml

    from ..api.crd import crd_manifest

    print(yaml.safe_dump(crd_manifest(), sort_keys=False))
    return 0


def _free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def cmd_bench(args):
    """bench.py (BASELINE metric contract) at one world size or a sweep:
    N = 1 runs it directly, N > 1 under ``torch.distributed.run`` (one rank
    per GPU, rendezvous on 127.0.0.1) -- the driver's launch lines.  Each run
    is a child process; its JSON line is printed, and for a sweep a table of
    aggregate / per-GPU throughput and weak-scaling efficiency against the
    smallest N follows."""
    import json
    import subprocess

    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    bench = os.path.join(root, "bench.py")
    if not os.path.exists(bench):
        print(f"pto bench: {bench} not found (run from a source checkout)", file=sys.stderr)
        return 2
    sizes = [int(x) for x in args.scale.split(",")] if args.scale else [args.gpus]
    extra = [a for a in (args.bench_args or []) if a != "--"]
    rows = []
    for n in sizes:
        if n == 1:
            cmd = [sys.executable, bench, "--gpus", "1"] + extra
        else:
            cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
                   "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", bench, "--gpus", str(n)] + extra
        r = subprocess.run(cmd, capture_output=True, text=True)
        lines = [ln for ln in r.stdout.splitlines() if ln.startswith('{"metric"')]
        if r.returncode != 0 or not lines:
            print(f"pto bench: N={n} failed (exit {r.returncode})\n{r.stderr[-2000:]}", file=sys.stderr)
            return r.returncode or 1
        print(lines[-1], flush=True)
        rows.append(json.loads(lines[-1]))
    if len(rows) > 1:
        base = rows[0]["value"] / rows[0]["n_gpus"]
        print(f"{'N':>3} {'value':>14} {'per GPU':>12} {'ms/step':>9} {'efficiency':>10}")
        for d in rows:
            per = d["value"] / d["n_gpus"]
            print(f"{d['n_gpus']:>3} {d['value']:>14,.1f} {per:>12,.1f} {d['ms_per_step']:>9.4f} {per / base:>10.1%}")
    return 0


def main(argv=None):
    p = argparse.ArgumentParser(prog="pto", description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument("--server", default=None, help="API server URL")
    p.add_argument("-n", "--namespace", default=None)
    sub = p.add_subparsers(dest="cmd", required=True)

    op = sub.add_parser("operator", help="run the PyTorchJob operator")
    add_operator_flags(op)
    op.set_defaults(fn=cmd_operator)

    ap = sub.add_parser("apiserver", help="run the API server")
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=8080)
    ap.add_argument("--wal", default=None, help="write-ahead log path for durability")
    ap.add_argument("--token", default=None)
    ap.set_defaults(fn=cmd_apiserver)

    nd = sub.add_parser("node", help="run the node manager + native agent")
    nd.add_argument("--gpus", "--gpus-per-node", dest="gpus", type=int, default=None,
                    help="GPUs managed by this node (default: all visible)")
    nd.add_argument("--hbm-per-gpu", default="288G", help="HBM per GPU for amd.com/hbm admission (quantity)")
    nd.add_argument("--node-agent-socket", default=None,
                    help="attach to a running pto-node-agent on this Unix socket instead of spawning one")
    nd.add_argument("--log-dir", default=None)
    nd.add_argument("--gpu-visibility", choices=["node", "isolated"], default=None,
                    help="node: replicas see every GPU and pick theirs via LOCAL_RANK (peer IPC/P2P reachable); "
                         "isolated: HIP_VISIBLE_DEVICES = the replica's own GPUs (default: $PTO_GPU_VISIBILITY or "
                         "isolated); a pod overrides it with the pto.amd.com/gpu-visibility annotation")
    nd.add_argument("--monitoring-port", type=int, default=0,
                    help="serve the pytorchjob_* training/HBM gauges on this port (0: off)")
    nd.add_argument("--node-name", default="mi355x-0")
    nd.add_argument("--master", default="")
    nd.set_defaults(fn=cmd_node)

    up = sub.add_parser("up", help="all-in-one single-node cluster")
    up.add_argument("--port", type=int, default=8080)
    up.add_argument("--gpus", "--gpus-per-node", dest="gpus", type=int, default=None)
    up.add_argument("--hbm-per-gpu", default="288G", help="HBM per GPU for amd.com/hbm admission (quantity)")
    up.add_argument("--wal", default=None)
    up.add_argument("--log-dir", default=None)
    up.add_argument("--monitoring-port", type=int, default=8443)
    up.add_argument("--enable-gang-scheduling", action="store_true")
    up.add_argument("--gpu-visibility", choices=["node", "isolated"], default=None,
                    help="GPU pinning model (see pto node --help)")
    up.add_argument("--restart-scope", choices=["job", "pod"], default="job",
                    help="ExitCode restarts of multi-replica jobs (see pto operator --help)")
    up.set_defaults(fn=cmd_up)

    a = sub.add_parser("apply")
    a.add_argument("-f", "--filename", required=True)
    a.set_defaults(fn=cmd_apply)

    g = sub.add_parser("get")
    g.add_argument("resource")
    g.add_argument("name", nargs="?")
    g.add_argument("-o", "--output", choices=["table", "json", "yaml"], default="table")
    g.add_argument("-A", "--all-namespaces", action="store_true")
    g.set_defaults(fn=cmd_get)

    d = sub.add_parser("describe")
    d.add_argument("name")
    d.set_defaults(fn=cmd_describe)

    lg = sub.add_parser("logs")
    lg.add_argument("name")
    lg.add_argument("--follow", "-f", action="store_true")
    lg.add_argument("--all", action="store_true", help="all replicas, not only the master")
    lg.set_defaults(fn=cmd_logs)

    de = sub.add_parser("delete")
    de.add_argument("resource", nargs="?", default="pytorchjobs")
    de.add_argument("name")
    de.set_defaults(fn=cmd_delete)

    w = sub.add_parser("watch")
    w.add_argument("name", nargs="?")
    w.add_argument("--timeout", type=int, default=600)
    w.set_defaults(fn=cmd_watch)

    cr = sub.add_parser("crd", help="print the CRD manifest")
    cr.set_defaults(fn=cmd_crd)

    bn = sub.add_parser("bench", help="run bench.py at one world size or a scaling sweep (e.g. --scale 1,2,4,8)")
    bn.add_argument("--gpus", type=int, default=1)
    bn.add_argument("--scale", default=None, help="comma-separated world sizes")
    bn.add_argument("bench_args", nargs=argparse.REMAINDER, help="passed to bench.py (e.g. -- --steps 200 --cpu)")
    bn.set_defaults(fn=cmd_bench)

    v = sub.add_parser("version")
    v.set_defaults(fn=lambda a: print(version_string()) or 0)

    args = p.parse_args(argv)
    return args.fn(args)


if __name__ == "__main__":
    sys.exit(main())
