"""Kubernetes cloud formation: pods of a StatefulSet find each other through
a headless service and start one torch.distributed rank per GPU.

Reference: h2o-k8s (water/k8s/H2OCluster.java, lookup/KubernetesDnsLookup.java,
lookup/{ClusterSize,Timeout}Constraint.java, api/KubernetesRestApi.java +
probe/KubernetesLeaderNodeProbeHandler.java).  The reference resolves the
headless service's DNS records until H2O_NODE_EXPECTED_COUNT pods answer (or
H2O_NODE_LOOKUP_TIMEOUT seconds pass), feeds the IPs to its flatfile
clustering and serves /kubernetes/isLeaderNode on port 8080 (or
H2O_KUBERNETES_API_PORT) so only the leader pod is marked ready.

Here the same environment contract yields a torchrun rendezvous instead of
a JVM flatfile: the pod IPs, sorted numerically, give every pod its node
rank; the lowest IP is the leader and the MASTER_ADDR; each pod then starts
`torch.distributed.run --nnodes N --nproc-per-node G --node-rank R` as a
CHILD process (the launcher itself never touches the GPU) and exits with
its code.  `deploy/helm/h2o3-amd` is the matching chart.

Usage inside a pod:  python -m h2o3_amd.parallel.k8s -- my_job.py --args
"""
from __future__ import annotations

import ipaddress
import os
import socket
import subprocess
import sys
import threading
import time
from http.server import BaseHTTPRequestHandler, HTTPServer

SERVICE_DNS_ENV = "H2O_KUBERNETES_SERVICE_DNS"
LOOKUP_TIMEOUT_ENV = "H2O_NODE_LOOKUP_TIMEOUT"
EXPECTED_COUNT_ENV = "H2O_NODE_EXPECTED_COUNT"
API_PORT_ENV = "H2O_KUBERNETES_API_PORT"
GPUS_ENV = "H2O3_GPUS_PER_POD"
MASTER_PORT_ENV = "H2O3_MASTER_PORT"


def is_running_on_kubernetes(env=None) -> bool:
    """KubernetesDnsLookup.isLookupPossible: the service DNS variable is set."""
    return SERVICE_DNS_ENV in (env if env is not None else os.environ)


def _resolve(name: str) -> set[str]:
    """IPv4/IPv6 addresses behind a headless service name (one A/AAAA record
    per ready pod)."""
    out = set()
    for fam, _, _, _, sa in socket.getaddrinfo(name, None, proto=socket.IPPROTO_TCP):
        if fam in (socket.AF_INET, socket.AF_INET6):
            out.add(sa[0])
    return out


def lookup_nodes(service_dns: str, expected: int | None = None, timeout_s: float | None = None,
                 resolver=_resolve, sleep=time.sleep, clock=time.monotonic, log=None) -> list[str]:
    """Resolve the service until `expected` pods are known or `timeout_s`
    passed (the reference's ClusterSizeConstraint / TimeoutConstraint: the
    lookup ends when EITHER constraint is met; with neither set, after the
    first successful lookup).  Returns the pod IPs sorted numerically."""
    if not service_dns or not service_dns.strip():
        raise ValueError(f"DNS Service '{service_dns}' name is invalid.")
    seen: set[str] = set()
    t0 = clock()
    while True:
        try:
            new = set(resolver(service_dns)) - seen
            for ip in sorted(new, key=_ip_key):
                if log:
                    log(f"New H2O pod with DNS record '{ip}' discovered.")
            seen |= new
        except OSError as e:   # NXDOMAIN while the first pods start, transient resolver errors
            if log:
                log(f"lookup of {service_dns} failed: {e}")
        done_size = expected is not None and len(seen) >= expected
        done_time = timeout_s is not None and clock() - t0 >= timeout_s
        if done_size or done_time or (expected is None and timeout_s is None and seen):
            break
        sleep(1.0)
    return sorted(seen, key=_ip_key)


def _ip_key(ip: str):
    a = ipaddress.ip_address(ip)
    return (a.version, int(a))


def own_ip(env=None) -> str:
    """This pod's IP: POD_IP (downward API, set by the chart), else the
    address the hostname resolves to."""
    env = env if env is not None else os.environ
    if env.get("POD_IP"):
        return env["POD_IP"]
    return socket.gethostbyname(socket.gethostname())


def node_plan(ips: list[str], me: str) -> dict:
    """Rank layout for the resolved pods: leader = lowest IP = MASTER_ADDR."""
    if me not in ips:
        raise RuntimeError(f"this pod's IP {me} is not among the service's pods {ips}")
    return {"nnodes": len(ips), "node_rank": ips.index(me), "master_addr": ips[0], "leader": ips.index(me) == 0}


def torchrun_cmd(plan: dict, nproc_per_node: int, script_args: list[str], master_port: int = 29500,
                 python: str = sys.executable) -> list[str]:
    return [python, "-m", "torch.distributed.run", f"--nnodes={plan['nnodes']}",
            f"--nproc-per-node={nproc_per_node}", f"--node-rank={plan['node_rank']}",
            f"--master-addr={plan['master_addr']}", f"--master-port={master_port}"] + list(script_args)


class _ProbeHandler(BaseHTTPRequestHandler):
    leader = False

    def do_GET(self):  # noqa: N802 - http.server API
        if self.path.rstrip("/") == "/kubernetes/isLeaderNode":
            code = 200 if self.leader else 404
        else:
            code = 404
        self.send_response(code)
        self.send_header("Content-Length", "0")
        self.end_headers()

    def log_message(self, *a):
        pass


def start_probe_api(leader: bool, port: int | None = None) -> HTTPServer:
    """KubernetesRestApi: /kubernetes/isLeaderNode answers 200 on the leader
    pod only (the chart's readiness probe), in a daemon thread."""
    port = int(port if port is not None else os.environ.get(API_PORT_ENV, 8080))
    handler = type("ProbeHandler", (_ProbeHandler,), {"leader": leader})
    srv = HTTPServer(("0.0.0.0", port), handler)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    return srv


def _gpus_per_pod(env) -> int:
    if env.get(GPUS_ENV):
        return int(env[GPUS_ENV])
    import torch
    return max(1, torch.cuda.device_count())   # counting devices does not initialise the GPU


def main(argv=None, env=None) -> int:
    env = env if env is not None else os.environ
    argv = list(sys.argv[1:] if argv is None else argv)
    if "--" in argv:
        argv = argv[argv.index("--") + 1:]
    if not argv:
        print("usage: python -m h2o3_amd.parallel.k8s -- script.py [args]", file=sys.stderr)
        return 2
    svc = env.get(SERVICE_DNS_ENV)
    if svc is None:
        raise SystemExit(f"DNS of H2O service not set. Please set the '{SERVICE_DNS_ENV}' variable.")
    timeout = float(env[LOOKUP_TIMEOUT_ENV]) if env.get(LOOKUP_TIMEOUT_ENV) else None
    expected = int(env[EXPECTED_COUNT_ENV]) if env.get(EXPECTED_COUNT_ENV) else None
    ips = lookup_nodes(svc, expected, timeout, log=lambda m: print(m, file=sys.stderr, flush=True))
    plan = node_plan(ips, own_ip(env))
    print(f"Using the following pods to form the cloud: [{','.join(ips)}] (node rank {plan['node_rank']})",
          file=sys.stderr, flush=True)
    start_probe_api(plan["leader"])
    cmd = torchrun_cmd(plan, _gpus_per_pod(env), argv, int(env.get(MASTER_PORT_ENV, 29500)))
    return subprocess.call(cmd, env=dict(env, HSA_ENABLE_IPC_MODE_LEGACY=env.get("HSA_ENABLE_IPC_MODE_LEGACY", "0")))


if __name__ == "__main__":
    sys.exit(main())
