"""Records longer than chunk_bytes on the GPU paths (reference behaviour: the
InputSplit buffer doubles until the record fits, src/io/input_split_base.cc:
241-258): a LibSVM line and a RecordIO record of 3 x chunk_bytes, zero-copy
on and off, equal the CPU output; the parser's slots grow instead of failing."""
import numpy as np
import pytest

import pyref
from dmlc_core_amd import data, io

pytestmark = pytest.mark.gpu

CHUNK = 64 * 1024


def _long_line(n_feat, seed):
    rng = np.random.default_rng(seed)
    idx = np.sort(rng.choice(1 << 24, n_feat, replace=False))
    return "1 " + " ".join(f"{i}:{rng.random():.6f}" for i in idx)


@pytest.mark.parametrize("zero_copy", [0, 1])
@pytest.mark.parametrize("hbm_cache", [0, 1])
def test_libsvm_line_of_three_chunks(tmp_path, zero_copy, hbm_cache):
    p = str(tmp_path / "l.libsvm")
    data.write_synthetic(p, 0, 800, seed=3)
    line = _long_line(12000, 1)  # ~ 200 KB > 3 x 64 KiB
    assert len(line) > 3 * CHUNK
    tail = str(tmp_path / "t.libsvm")
    data.write_synthetic(tail, 800, 1600, seed=3)
    with open(p, "a") as f:
        f.write(line + "\n" + open(tail).read())
    cpu = pyref.concat_blocks(list(data.iter_blocks(p, type="libsvm")))
    g = data.GPUParser(p, chunk_bytes=CHUNK, zero_copy=zero_copy, hbm_cache=hbm_cache)
    for _ in range(2 if hbm_cache else 1):
        g.before_first()
        got = pyref.concat_blocks([g.parse_all().to_host()])
        for k in ("label", "offset", "index", "value"):
            np.testing.assert_array_equal(got[k], cpu[k], err_msg=k)
    g.before_first()
    blocks = []
    while g.next():
        blocks.append(g.value_to_host())
    got = pyref.concat_blocks(blocks)
    np.testing.assert_array_equal(got["index"], cpu["index"])


@pytest.mark.parametrize("zero_copy", [0, 1])
def test_recordio_record_of_three_chunks(tmp_path, zero_copy):
    rng = np.random.default_rng(5)
    recs = [bytes(rng.integers(0, 256, int(rng.integers(0, 900)), dtype=np.uint8))
            for _ in range(400)]
    recs.insert(200, bytes(rng.integers(0, 256, 3 * CHUNK + 123, dtype=np.uint8)))
    p = str(tmp_path / "r.rec")
    w = io.RecordIOWriter(p)
    for r in recs:
        w.write(r)
    w.close()
    r = io.GPURecordIO(p, chunk_bytes=CHUNK, zero_copy=zero_copy)
    r.read_all()
    off, payload = r.resident_to_host()
    assert io.split_records(off, payload) == recs
