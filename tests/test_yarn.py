"""YARN: the dmlc ApplicationMaster policy (reference
tracker/yarn/.../ApplicationMaster.java:482-610) over local process
containers, and the JVM-free Services REST submission against a mock RM."""
import json
import os
import sys
import threading
import urllib.parse
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

import pytest

from dmlc_core_amd.parallel.launch import yarn
import yarn_am_sim as yarn_am
from dmlc_core_amd.parallel.launch.opts import get_opts

PY = sys.executable


def _task_cmd(tmp_path, body):
    script = tmp_path / "task.py"
    script.write_text("import os, sys\n" + body)
    return [PY, str(script)]


def test_am_runs_every_task_once_with_dmlc_env(tmp_path):
    out = tmp_path / "out"
    out.mkdir()
    cmd = _task_cmd(tmp_path, f"open(os.path.join({str(out)!r}, os.environ['DMLC_TASK_ID']), 'w')"
                              ".write(os.environ['DMLC_ROLE'] + ' ' + os.environ['DMLC_NODE_HOST'] + ' '"
                              " + os.environ['DMLC_NUM_ATTEMPT'] + ' ' + os.environ['DMLC_TRACKER_URI'])\n")
    be = yarn_am.LocalContainerBackend(nodes=["n0", "n1"])
    env = {"DMLC_NUM_WORKER": "3", "DMLC_NUM_SERVER": "1", "DMLC_TRACKER_URI": "10.0.0.1",
           "DMLC_WORKER_MEMORY_MB": "2048", "OTHER": "x"}
    am = yarn_am.ApplicationMaster.from_env(be, cmd, env)
    assert am.res["worker"].memory_mb == 2048
    res = am.run(timeout=60)
    assert res.success and res.finished == 4 and res.failed == 0
    got = {int(p.name): p.read_text().split() for p in out.iterdir()}
    assert sorted(got) == [0, 1, 2, 3]
    assert [got[i][0] for i in range(4)] == ["worker", "worker", "worker", "server"]
    assert all(g[2] == "0" and g[3] == "10.0.0.1" for g in got.values())
    assert all("OTHER" not in e for _, _, e in be.launched)  # only DMLC_* is forwarded


def test_am_retries_on_another_node_and_blacklists(tmp_path):
    """Every container on n0 fails: the task is retried (attempt 1), n0 is
    blacklisted, later n0 containers are released unused, the job succeeds."""
    cmd = _task_cmd(tmp_path, "sys.exit(0)\n")
    be = yarn_am.LocalContainerBackend(nodes=["n0", "n1", "n2"], fail_nodes={"n0": 1})
    am = yarn_am.ApplicationMaster(be, cmd, num_worker=3, max_attempt=3, env={})
    res = am.run(timeout=60)
    assert res.success, res.diagnostics
    assert res.blacklist == ["n0"]
    assert res.attempts[0] == 1 and res.attempts[1] == 0 and res.attempts[2] == 0
    assert be.released  # a later allocation on n0 was handed back
    retried = [e for _, node, e in be.launched if e["DMLC_TASK_ID"] == "0"]
    assert [e["DMLC_NUM_ATTEMPT"] for e in retried] == ["0", "1"]


def test_am_aborts_after_max_attempts(tmp_path):
    cmd = _task_cmd(tmp_path, "sys.exit(int(os.environ['DMLC_TASK_ID'] == '1') * 3)\n")
    be = yarn_am.LocalContainerBackend(nodes=[f"n{i}" for i in range(8)])
    am = yarn_am.ApplicationMaster(be, cmd, num_worker=2, max_attempt=2, env={})
    res = am.run(timeout=60)
    assert not res.success
    assert "Task 1 failed more than 2 times" in res.diagnostics
    assert res.finished == 1 and res.failed == 1
    assert res.diagnostics.startswith("Diagnostics., num_tasks2, finished=1, failed=1")


@pytest.mark.parametrize("status,word", [(yarn_am.KILLED_EXCEEDED_PMEM, "physical"),
                                         (yarn_am.KILLED_EXCEEDED_VMEM, "virtual")])
def test_am_memory_kill_aborts_immediately(tmp_path, status, word):
    cmd = _task_cmd(tmp_path, "import time; time.sleep(30)\n")
    be = yarn_am.LocalContainerBackend(nodes=["bad", "ok1", "ok2"], fail_nodes={"bad": status})
    am = yarn_am.ApplicationMaster(be, cmd, num_worker=3, max_attempt=5, env={})
    res = am.run(timeout=60)
    assert not res.success
    assert f"exceeding allocated {word} memory" in res.diagnostics
    assert res.failed == 3 and res.finished == 0  # the sleeping tasks were stopped
    assert not be.procs


# ------------------------------------------------------------ Services REST API
class _RM(BaseHTTPRequestHandler):
    protocol_version = "HTTP/1.1"
    services = {}
    script = []  # successive container states returned by GET
    deleted = []

    def log_message(self, *a):
        pass

    def _send(self, code, obj=None):
        b = json.dumps(obj).encode() if obj is not None else b""
        self.send_response(code)
        self.send_header("Content-Length", str(len(b)))
        self.end_headers()
        self.wfile.write(b)

    def do_POST(self):
        n = int(self.headers["Content-Length"])
        spec = json.loads(self.rfile.read(n))
        assert urllib.parse.urlsplit(self.path).query == "user.name=alice"
        self.services[spec["name"]] = spec
        self._send(202, {"uri": "/app/v1/services/" + spec["name"]})

    def do_GET(self):
        name = urllib.parse.urlsplit(self.path).path.rsplit("/", 1)[1]
        st = self.script.pop(0) if len(self.script) > 1 else self.script[0]
        self._send(200, dict(st, name=name))

    def do_DELETE(self):
        self.deleted.append(urllib.parse.urlsplit(self.path).path.rsplit("/", 1)[1])
        self._send(200, {})


@pytest.fixture()
def rm():
    srv = ThreadingHTTPServer(("127.0.0.1", 0), _RM)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    _RM.services, _RM.deleted = {}, []
    os.environ["HADOOP_USER_NAME"] = "alice"
    yield f"http://127.0.0.1:{srv.server_address[1]}"
    os.environ.pop("HADOOP_USER_NAME", None)
    srv.shutdown()


def _args(*extra):
    return get_opts(["--cluster", "yarn", "--num-workers", "4", "--num-servers", "1",
                     "--worker-memory", "2g", "--gpus-per-node", "8", "--env", "FOO=bar",
                     *extra, "python", "train.py"])


def test_service_spec_shapes_components():
    spec = yarn.service_spec(_args(), {"DMLC_TRACKER_URI": "1.2.3.4", "DMLC_TRACKER_PORT": 9091},
                             "job")
    comps = {c["name"]: c for c in spec["components"]}
    w, s = comps["worker"], comps["server"]
    assert w["number_of_containers"] == 4 and s["number_of_containers"] == 1
    # one rank per container: one GPU each, never --gpus-per-node of them
    assert w["resource"]["memory"] == "2048" and w["resource"]["additional"]["amd.com/gpu"]["value"] == 1
    assert "additional" not in s["resource"]
    assert w["configuration"]["env"]["DMLC_TRACKER_PORT"] == "9091"
    assert w["configuration"]["env"]["DMLC_ROLE"] == "worker" and w["configuration"]["env"]["FOO"] == "bar"
    assert w["launch_command"].endswith("python train.py")


@pytest.mark.parametrize("instance,role", [(0, "worker"), (3, "worker"), (0, "server")])
def test_service_containers_get_their_own_identity(instance, role):
    """Every container derives its own DMLC_TASK_ID (workers 0..n-1, servers
    after them, as the reference AM numbers tasks) and DMLC_NODE_HOST from
    the service's ${COMPONENT_ID}; GPU workers bind local rank 0.  The launch
    command is run through bash with the placeholder expanded as the YARN
    service does."""
    import subprocess
    spec = yarn.service_spec(_args(), {}, "job")
    comp = {c["name"]: c for c in spec["components"]}[role]
    cmd = comp["launch_command"].replace("${COMPONENT_ID}", str(instance))
    cmd = cmd[:cmd.rindex("python train.py")] + \
        'echo "$DMLC_TASK_ID ${DMLC_LOCAL_RANK:-none} $DMLC_NODE_HOST"'
    out = subprocess.run(["bash", "-c", cmd], capture_output=True, text=True, check=True).stdout
    tid, local, host = out.split()
    assert int(tid) == (instance if role == "worker" else 4 + instance)
    assert local == ("0" if role == "worker" else "none")
    assert host


def test_service_containers_count_their_attempts(tmp_path):
    """A relaunched container (same instance) exports DMLC_NUM_ATTEMPT 1, 2,
    ... from the tracker's launch count of its task id, as the reference AM
    does per launch; without a tracker the first attempt, 0"""
    import subprocess
    from dmlc_core_amd.parallel import tracker as trk
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = yarn.service_spec(_args(), {}, "job")
    comp = {c["name"]: c for c in spec["components"]}["worker"]
    cmd = comp["launch_command"].replace("${COMPONENT_ID}", "2")
    cmd = cmd[:cmd.rindex("python train.py")] + 'echo "$DMLC_TASK_ID $DMLC_NUM_ATTEMPT"'
    env = dict(os.environ, PYTHONPATH=repo, DMLC_ROLE="worker")
    env.pop("DMLC_TRACKER_URI", None)
    run = lambda e: subprocess.run(["bash", "-c", cmd], capture_output=True, text=True,  # noqa: E731
                                   check=True, env=e, cwd=str(tmp_path)).stdout.split()
    assert run(env) == ["2", "0"]
    t = trk.RabitTracker("127.0.0.1", 1, port=19500, port_end=19999, timeout=60)
    t.start(1)
    try:
        env.update(DMLC_TRACKER_URI="127.0.0.1", DMLC_TRACKER_PORT=str(t.port))
        assert [run(env) for _ in range(3)] == [["2", "0"], ["2", "1"], ["2", "2"]]
    finally:
        t.stop()


def test_service_job_success_and_memory_abort(rm):
    job = yarn.YarnServiceJob(rm, "j1")
    job.submit(yarn.service_spec(_args(), {}, "j1"))
    assert "j1" in _RM.services
    _RM.script = [{"state": "ACCEPTED"}, {"state": "STARTED", "components": []},
                  {"state": "SUCCEEDED"}]
    assert job.wait(poll=0.01) == (True, "SUCCEEDED")
    # a container killed by the NM memory monitor aborts the service at once
    _RM.script = [{"state": "STARTED", "components": [{"name": "worker", "containers": [
        {"id": "c1", "state": "FAILED",
         "diagnostics": "Container is running 2.1GB beyond physical memory limits"}]}]}]
    ok, diag = job.wait(poll=0.01)
    assert not ok and "exceeding allocated memory" in diag and _RM.deleted == ["j1"]


def test_service_job_aborts_after_repeated_failures(rm):
    job = yarn.YarnServiceJob(rm, "j2")
    def failed(cid):
        return {"state": "STARTED", "components": [{"name": "worker", "containers": [
            {"id": cid, "component_instance_name": "worker-0", "state": "FAILED",
             "diagnostics": "exit 1"}]}]}
    # the same failed container seen on several polls counts once
    _RM.script = [failed("c7"), failed("c7"), failed("c8"), failed("c8"), failed("c9")]
    ok, diag = job.wait(poll=0.01, max_attempt=3)
    assert not ok and "worker/worker-0 failed more than 3 times" in diag
    assert _RM.deleted == ["j2"]


def test_submit_dry_run_uses_services_api_without_jar(monkeypatch, capsys):
    """With YARN_RM_ADDRESS set and no dmlc-yarn.jar, dmlc-submit --cluster
    yarn builds a Services spec instead of a hadoop jar command."""
    monkeypatch.setenv("YARN_RM_ADDRESS", "http://rm.invalid:8088")
    monkeypatch.delenv("DMLC_YARN_APP_DIR", raising=False)
    assert yarn.submit(_args("--dry-run")) == 0
    spec = json.loads(capsys.readouterr().out)
    assert {c["name"] for c in spec["components"]} == {"worker", "server"}
    assert spec["queue"] == "default"


def test_service_stages_files_and_archives_through_webhdfs(rm, tmp_path, monkeypatch):
    """-file / -archive shipping (reference Client.java:122-160) on the
    Services path: payloads go through the native WebHDFS backend (namenode
    redirect -> datanode, no body to the namenode) into the staging dir, and
    every component localises them (STATIC files, ARCHIVE unpacked)."""
    import tarfile

    import mock_remote
    mock_remote.WebHdfsHandler.store = {}
    mock_remote.WebHdfsHandler.namenode_bodies = 0
    srv = mock_remote.serve(mock_remote.WebHdfsHandler)
    try:
        addr = f"127.0.0.1:{srv.server_address[1]}"
        monkeypatch.setenv("DMLC_YARN_STAGING", f"webhdfs://{addr}/user/alice/.dmlc/")
        script = tmp_path / "train_job.py"
        script.write_text("print('hi')\n")
        blob = tmp_path / "vocab.bin"
        blob.write_bytes(bytes(range(256)) * 4096)
        (tmp_path / "env").mkdir()
        (tmp_path / "env" / "cfg.txt").write_text("x=1\n")
        arc = tmp_path / "env.tar.gz"
        with tarfile.open(arc, "w:gz") as t:
            t.add(tmp_path / "env", arcname="env")
        args = get_opts(["--cluster", "yarn", "--num-workers", "2", "--files", str(blob),
                         "--archives", str(arc), "python", str(script), "--epochs", "3"])
        entries = yarn.stage_files(args, "job-7")
        job = yarn.YarnServiceJob(rm, "job-7")
        job.submit(yarn.service_spec(args, {}, "job-7", entries))
        store = mock_remote.WebHdfsHandler.store
        base = "/user/alice/.dmlc/job-7/"
        assert store[base + "train_job.py"] == script.read_bytes()
        assert store[base + "vocab.bin"] == blob.read_bytes()
        assert store[base + "env.tar.gz"] == arc.read_bytes()
        assert mock_remote.WebHdfsHandler.namenode_bodies == 0
        comp = _RM.services["job-7"]["components"][0]
        files = {f["dest_file"]: f for f in comp["configuration"]["files"]}
        assert files["train_job.py"] == {"type": "STATIC", "src_file": base + "train_job.py",
                                         "dest_file": "train_job.py"}
        assert files["vocab.bin"]["type"] == "STATIC"
        assert files["env.tar.gz"] == {"type": "ARCHIVE", "src_file": base + "env.tar.gz",
                                       "dest_file": "env.tar.gz"}
        assert comp["launch_command"].endswith("; python ./train_job.py --epochs 3")
        assert comp["configuration"]["env"]["DMLC_JOB_ARCHIVES"] == "env.tar.gz"
    finally:
        srv.shutdown()


def test_service_staging_requires_a_target(monkeypatch, tmp_path):
    monkeypatch.delenv("DMLC_YARN_STAGING", raising=False)
    monkeypatch.delenv("DMLC_WEBHDFS_ENDPOINT", raising=False)
    f = tmp_path / "a.txt"
    f.write_text("1")
    args = get_opts(["--cluster", "yarn", "--num-workers", "1", "--files", str(f), "true"])
    with pytest.raises(SystemExit, match="DMLC_YARN_STAGING"):
        yarn.stage_files(args, "j")
    monkeypatch.setenv("DMLC_WEBHDFS_ENDPOINT", "http://nn:9870")
    assert yarn.staging_root(args) == "webhdfs://nn:9870/tmp"
    assert yarn.stage_files(args, "j", upload=False)[0]["src_file"] == "/tmp/j/a.txt"


def test_service_job_blacklists_failed_nodes(rm):
    """a failed container's node is blacklisted: the spec asks the service AM
    to exclude it (node-blacklist threshold 1, as the reference AM's
    updateBlacklist on each failure), and a retry placed on it anyway counts
    as a failed attempt of that task"""
    spec = yarn.service_spec(_args(), {}, "j3")
    for comp in spec["components"]:
        assert comp["configuration"]["properties"]["yarn.service.node-blacklist.threshold"] == "1"
    job = yarn.YarnServiceJob(rm, "j3")
    job.submit(spec)

    def st(*cs):
        return {"state": "STARTED", "components": [{"name": "worker", "containers": list(cs)}]}
    fail_a = {"id": "c1", "component_instance_name": "worker-0", "state": "FAILED",
              "bare_host": "nodeA", "diagnostics": "exit 1"}
    on_b = {"id": "c2", "component_instance_name": "worker-0", "state": "READY", "bare_host": "nodeB"}
    _RM.script = [st(fail_a), st(fail_a, on_b), {"state": "SUCCEEDED"}]
    assert job.wait(poll=0.01, max_attempt=3) == (True, "SUCCEEDED")
    assert job.blacklist == {"nodeA"}
    # re-placed on the blacklisted node, twice: the attempts run out
    on_a = [{"id": f"c{i}", "component_instance_name": "worker-0", "state": "READY",
             "bare_host": "nodeA"} for i in (3, 4)]
    _RM.script = [st(fail_a), st(fail_a, on_a[0]), st(fail_a, on_a[1])]
    ok, diag = job.wait(poll=0.01, max_attempt=3)
    assert not ok and "blacklisted node nodeA" in diag


def test_service_job_does_not_penalise_a_container_placed_before_its_node_was_blacklisted(rm):
    """worker-0 fails on nodeX and restarts on nodeY; later worker-1 fails on
    nodeY, which blacklists it.  worker-0's healthy retry on nodeY was placed
    before that and must not count as a failed attempt (max_attempt 2 would
    abort the job if it did)"""
    job = yarn.YarnServiceJob(rm, "j4")
    job.submit(yarn.service_spec(_args(), {}, "j4"))

    def st(*cs):
        return {"state": "STARTED", "components": [{"name": "worker", "containers": list(cs)}]}
    w0_fail = {"id": "c1", "component_instance_name": "worker-0", "state": "FAILED",
               "bare_host": "nodeX", "diagnostics": "exit 1"}
    w0_retry = {"id": "c2", "component_instance_name": "worker-0", "state": "READY",
                "bare_host": "nodeY"}
    w1_fail = {"id": "c3", "component_instance_name": "worker-1", "state": "FAILED",
               "bare_host": "nodeY", "diagnostics": "exit 1"}
    w1_retry = {"id": "c4", "component_instance_name": "worker-1", "state": "READY",
                "bare_host": "nodeZ"}
    _RM.script = [st(w0_fail), st(w0_fail, w0_retry), st(w0_fail, w0_retry, w1_fail),
                  st(w0_fail, w0_retry, w1_fail, w1_retry), {"state": "SUCCEEDED"}]
    assert job.wait(poll=0.01, max_attempt=2) == (True, "SUCCEEDED")
    assert job.blacklist == {"nodeX", "nodeY"}


def test_submit_without_a_resourcemanager_explains_the_services_path(monkeypatch):
    """there is no `hadoop jar` mode: --cluster yarn needs YARN_RM_ADDRESS"""
    monkeypatch.delenv("YARN_RM_ADDRESS", raising=False)
    with pytest.raises(SystemExit, match="YARN_RM_ADDRESS"):
        yarn.submit(_args())
