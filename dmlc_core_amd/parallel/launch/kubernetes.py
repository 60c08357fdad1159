"""Kubernetes backend (reference `tracker/dmlc_tracker/kubernetes.py:30-143`):
a Job + headless Service per role (scheduler / server / worker), optional
YAML templates, ``restartPolicy: OnFailure``.  Manifests are plain dicts
applied with ``kubectl apply -f -`` (no kubernetes Python client needed --
the reference hard-imported it, §7.4 #6).  Workers request
``amd.com/gpu: --gpus-per-node`` and bind by JOB_COMPLETION_INDEX.
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


def manifests(args, envs: Dict[str, object], cmd: str) -> List[dict]:
    job = (args.jobname or "dmlc").lower()
    out = []
    roles = [("worker", args.num_workers, args.kube_worker_image, args.kube_worker_template,
              args.worker_cores, args.worker_memory_mb, args.gpus_per_node)]
    if args.num_servers:
        roles.append(("server", args.num_servers, args.kube_server_image,
                      args.kube_server_template, args.server_cores, args.server_memory_mb, 0))
    for role, n, image, template, cores, mem, gpus in roles:
        env = dict(envs, DMLC_ROLE=role, DMLC_JOB_CLUSTER="kubernetes")
        body = cmd
        if role == "worker":
            body = ("export DMLC_TASK_ID=$JOB_COMPLETION_INDEX DMLC_WORKER_ID=$JOB_COMPLETION_INDEX; "
                    + (f"export DMLC_LOCAL_RANK=$((JOB_COMPLETION_INDEX % {gpus})); " if gpus else "")
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
        spec["spec"]["template"]["spec"]["containers"] = [
            _container(role, image, body, env, cores, mem, gpus if role == "worker" else 0)]
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
