"""In-container task launcher (reference `tracker/dmlc_tracker/launcher.py:18-81`).

Runs inside each scheduled task (SGE array job, YARN container): derives
DMLC_TASK_ID / DMLC_ROLE from the scheduler's task index, extends
LD_LIBRARY_PATH / CLASSPATH for libhdfs + the JVM when HADOOP_HOME /
JAVA_HOME are set, maps DMLC_HDFS_OPTS to LIBHDFS_OPTS, unpacks
DMLC_JOB_ARCHIVES, then runs the user command as a child process and exits
with its status.
"""
from __future__ import annotations

import glob
import os
import subprocess
import sys
import zipfile


def prepare_env(env: dict) -> dict:
    env = dict(env)
    if "SGE_TASK_ID" in env and "DMLC_TASK_ID" not in env:
        tid = int(env["SGE_TASK_ID"]) - 1
        nworker = int(env.get("DMLC_NUM_WORKER", "0"))
        env["DMLC_TASK_ID"] = str(tid if tid < nworker else tid - nworker)
        env["DMLC_ROLE"] = "worker" if tid < nworker else "server"
    libs = []
    hadoop = env.get("HADOOP_HOME") or env.get("HADOOP_PREFIX")
    java = env.get("JAVA_HOME")
    if hadoop:
        libs.append(os.path.join(hadoop, "lib", "native"))
        try:
            cp = subprocess.run([os.path.join(hadoop, "bin", "hadoop"), "classpath", "--glob"],
                                capture_output=True, text=True, timeout=60).stdout.strip()
            if cp:
                env["CLASSPATH"] = cp + (":" + env["CLASSPATH"] if env.get("CLASSPATH") else "")
        except (OSError, subprocess.SubprocessError):
            pass
    if java:
        libs += glob.glob(os.path.join(java, "jre", "lib", "amd64", "server")) + \
            glob.glob(os.path.join(java, "lib", "server"))
    if libs:
        env["LD_LIBRARY_PATH"] = ":".join(libs + [env.get("LD_LIBRARY_PATH", "")]).rstrip(":")
    if "DMLC_HDFS_OPTS" in env:
        env["LIBHDFS_OPTS"] = env["DMLC_HDFS_OPTS"]
    elif "LIBHDFS_OPTS" not in env:
        env["LIBHDFS_OPTS"] = "-Xmx128m"
    return env


def unpack_archives(env: dict) -> None:
    for a in filter(None, env.get("DMLC_JOB_ARCHIVES", "").split(":")):
        name = os.path.basename(a)
        if name.endswith(".zip") and os.path.exists(name):
            with zipfile.ZipFile(name) as z:
                z.extractall(name[:-4])


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    if not argv:
        print("usage: python -m dmlc_core_amd.parallel.launch.container <command...>", file=sys.stderr)
        return 2
    env = prepare_env(os.environ)
    unpack_archives(env)
    return subprocess.call(" ".join(argv), shell=True, env=env)


if __name__ == "__main__":
    sys.exit(main())
