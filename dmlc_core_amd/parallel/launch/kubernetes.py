"""Kubernetes backend (reference `tracker/dmlc_tracker/kubernetes.py:30-143`):
a Job + headless Service per role (scheduler / server / worker), optional
YAML templates, ``restartPolicy: OnFailure``.  Manifests are plain dicts
applied with ``kubectl apply -f -`` (no kubernetes Python client needed --
the reference hard-imported it, §7.4 #6).

GPU workers run one process per GPU.  With ``--gpus-per-node G`` the worker
Job has one pod per node (``ceil(num_workers / G)`` indexed pods), each
requesting ``amd.com/gpu: G`` and starting its ``min(G, rest)`` ranks itself
with ``DMLC_LOCAL_RANK`` = 0..G-1 and ``DMLC_TASK_ID`` = pod index x G +
local rank: the ranks of a node share one pod, so RCCL's peer-to-peer xGMI
paths (IPC between processes) work inside it.  ``--kube-pod-per-rank 1``
instead gives every rank its own pod with exactly one GPU (local rank 0 --
the device plugin exposes only that GPU to the pod); RCCL then uses the
network between pods.  No pod ever requests more GPUs than it runs ranks.
"""
from __future__ import annotations

import copy
import subprocess
from typing import Dict, List

import yaml

from .. import tracker
from .opts import user_envs


def _container(name, image, cmd, env, cores, mem_mb, gpus=0):
    res = {"cpu": str(cores), "memory": f"{mem_mb}Mi"}
    c = {"name": name, "image": image, "command": ["/bin/bash", "-c", cmd],
         "env": [{"name": k, "value": str(v)} for k, v in sorted(env.items())],
         "resources": {"requests": dict(res), "limits": dict(res)}}
    if gpus:
        c["resources"]["limits"]["amd.com/gpu"] = gpus
    return c


def _node_pod_body(cmd: str, gpus: int, nworker: int) -> str:
    """the command of a pod-per-node worker: starts this pod's ranks (one per
    GPU) in the background, each with its own task id and local rank, and
    exits with the first non-zero rank status"""
    return (f"G={gpus}; B=$((JOB_COMPLETION_INDEX * G)); R=$(({nworker} - B)); "
            "if [ $R -gt $G ]; then R=$G; fi; pids=''; "
            "for i in $(seq 0 $((R - 1))); do "
            "( export DMLC_LOCAL_RANK=$i LOCAL_RANK=$i LOCAL_WORLD_SIZE=$R "
            "DMLC_TASK_ID=$((B + i)) DMLC_WORKER_ID=$((B + i)); "
            + cmd + " ) & pids=\"$pids $!\"; done; "
            "rc=0; for p in $pids; do wait $p; s=$?; "
            "if [ $s -ne 0 ] && [ $rc -eq 0 ]; then rc=$s; fi; done; exit $rc")


def manifests(args, envs: Dict[str, object], cmd: str) -> List[dict]:
    job = (args.jobname or "dmlc").lower()
    out = []
    gpus = int(args.gpus_per_node or 0)
    per_rank = bool(getattr(args, "kube_pod_per_rank", False))
    nworker = int(args.num_workers)
    # worker pods and the GPUs each one requests: one per rank (1 GPU) or
    # one per node (G GPUs, G ranks)
    if gpus and not per_rank:
        wpods, wgpus = -(-nworker // gpus), min(gpus, nworker)
    else:
        wpods, wgpus = nworker, 1 if gpus else 0
    # a pod-per-node pod runs wgpus ranks: it gets each rank's cores / memory
    ranks_per_pod = wgpus if (gpus and not per_rank) else 1
    roles = [("worker", wpods, args.kube_worker_image, args.kube_worker_template,
              args.worker_cores * ranks_per_pod, args.worker_memory_mb * ranks_per_pod, wgpus)]
    if args.num_servers:
        roles.append(("server", args.num_servers, args.kube_server_image,
                      args.kube_server_template, args.server_cores, args.server_memory_mb, 0))
    for role, n, image, template, cores, mem, pod_gpus in roles:
        env = dict(envs, DMLC_ROLE=role, DMLC_JOB_CLUSTER="kubernetes")
        body = cmd
        if role == "worker":
            if gpus and not per_rank:
                body = _node_pod_body(cmd, wgpus, nworker)
            else:
                body = ("export DMLC_TASK_ID=$JOB_COMPLETION_INDEX "
                        "DMLC_WORKER_ID=$JOB_COMPLETION_INDEX; "
                        + ("export DMLC_LOCAL_RANK=0 LOCAL_RANK=0 LOCAL_WORLD_SIZE=1; "
                           if gpus else "")
                        + cmd)
        if template:
            with open(template) as f:
                spec = yaml.safe_load(f)
        else:
            spec = {"apiVersion": "batch/v1", "kind": "Job",
                    "metadata": {"name": f"{job}-{role}", "namespace": args.kube_namespace},
                    "spec": {"completions": n, "parallelism": n, "completionMode": "Indexed",
                             "template": {"metadata": {"labels": {"dmlc-job": job, "role": role}},
                                          "spec": {"restartPolicy": "OnFailure",
                                                   "subdomain": f"{job}-{role}",
                                                   "containers": []}}}}
        spec = copy.deepcopy(spec)
        spec["spec"]["completions"] = spec["spec"]["parallelism"] = n
        spec["spec"]["template"]["spec"]["containers"] = [
            _container(role, image, body, env, cores, mem, pod_gpus)]
        out.append(spec)
        out.append({"apiVersion": "v1", "kind": "Service",
                    "metadata": {"name": f"{job}-{role}", "namespace": args.kube_namespace},
                    "spec": {"clusterIP": "None", "selector": {"dmlc-job": job, "role": role}}})
    return out


def submit(args):
    cmd = " ".join(args.command)

    def launch(nworker, nserver, envs):
        envs = dict(envs)
        envs.update(user_envs(args))
        text = yaml.safe_dump_all(manifests(args, envs, cmd), sort_keys=False)
        if args.dry_run:
            print(text)
            return
        subprocess.run(["kubectl", "apply", "-f", "-"], input=text, text=True, check=True)

    if args.dry_run:
        launch(args.num_workers, args.num_servers, {"DMLC_NUM_WORKER": args.num_workers,
                                                    "DMLC_NUM_SERVER": args.num_servers})
        return 0
    tracker.submit(args.num_workers, args.num_servers, launch, host_ip=args.host_ip or "auto",
                   pscmd=cmd, timeout=args.timeout, heartbeat_timeout=args.heartbeat_timeout)
    return 0
