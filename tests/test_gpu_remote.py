"""BASELINE config 4: s3:// / http:// objects -> parallel ranged GETs into the
pinned-host ring -> hipMemcpyAsync -> HIP parse -> CSR in HBM.  The S3
endpoint is the in-process SigV4-verifying mock (no network); results must
be bit-identical to the same files parsed from local disk."""
import os

import numpy as np
import pytest

import mock_remote
import pyref
from dmlc_core_amd import data, io

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not os.path.exists("/usr/lib/x86_64-linux-gnu/libcurl.so.4"),
                                 reason="libcurl not installed")]


@pytest.fixture(scope="module")
def s3():
    srv = mock_remote.serve(mock_remote.S3Handler)
    os.environ.update({"S3_ENDPOINT": f"http://127.0.0.1:{srv.server_address[1]}",
                       "S3_ACCESS_KEY_ID": "AKIDTEST", "S3_SECRET_ACCESS_KEY": "secret",
                       "S3_REGION": "us-east-1", "DMLC_S3_WRITE_BUFFER_MB": "5"})
    yield mock_remote.S3Handler
    srv.shutdown()


def _upload(local_dir, prefix, nfiles, rows, fmt="libsvm"):
    for i in range(nfiles):
        f = local_dir / f"part-{i}.{fmt}"
        data.write_synthetic(str(f), i * rows, (i + 1) * rows, format=fmt, seed=9)
        w = io.Stream(f"{prefix}/part-{i}.{fmt}", "w")
        w.write(f.read_bytes())
        w.close()


@pytest.mark.parametrize("nparts", [1, 3])
def test_s3_gpu_parse_equals_local(s3, tmp_path, nparts):
    _upload(tmp_path, "s3://gpubk/train", 2, 20000)
    for part in range(nparts):
        cfg = dict(chunk_bytes=4 << 20, read_threads=4)
        remote = data.GPUParser("s3://gpubk/train", part, nparts, **cfg)
        assert not remote.stats()["zero_copy"]  # remote data always takes the pinned ring
        r = remote.parse_all().to_host()
        loc = data.GPUParser(str(tmp_path), part, nparts, zero_copy=0, **cfg).parse_all().to_host()
        for k in ("label", "offset", "index", "value"):
            np.testing.assert_array_equal(r[k], loc[k], err_msg=k)


def test_s3_gpu_recordio_equals_local(s3, tmp_path):
    f = tmp_path / "r.rec"
    data.write_synthetic(str(f), 0, 20000, format="recordio", seed=4, record_bytes=300)
    w = io.Stream("s3://gpubk/rec/r.rec", "w")
    w.write(f.read_bytes())
    w.close()
    a = io.GPURecordIO("s3://gpubk/rec/r.rec", 0, 2, chunk_mb=2)
    b = io.GPURecordIO(str(f), 0, 2, chunk_mb=2, zero_copy=0)
    a.read_all()
    b.read_all()
    oa, da = a.resident_to_host()
    ob, db = b.resident_to_host()
    np.testing.assert_array_equal(np.asarray(oa), np.asarray(ob))
    assert da == db
