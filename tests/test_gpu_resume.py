"""Mid-epoch resume of the GPU parser: stop after k streamed
blocks, checkpoint the cursor, restart a *new* parser (other ingest mode,
other chunk size) from it -- the union is bit-identical to one CPU pass."""
import numpy as np
import pytest

import pyref
from dmlc_core_amd import data

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("zc_first,zc_second", [(0, 1), (1, 0), (1, 1)])
def test_gpu_parser_resume_from_cursor(tmp_path, zc_first, zc_second):
    d = tmp_path / "ds"
    d.mkdir()
    for i in range(2):
        data.write_synthetic(str(d / f"p{i}.libsvm"), i * 6000, (i + 1) * 6000, seed=8)
    uri = str(d)
    cpu = pyref.concat_blocks(list(data.iter_blocks(uri, 0, 1, type="libsvm")))
    g = data.GPUParser(uri, chunk_bytes=512 << 10, zero_copy=zc_first)
    head = []
    for _ in range(3):
        assert g.next()
        head.append(g.value_to_host())
    state = g.state_dict()
    assert 0 < state["cursor"] < g.partition_bytes
    del g
    g2 = data.GPUParser(uri, chunk_bytes=300 << 10, zero_copy=zc_second)
    g2.load_state_dict(state)
    rest = g2.parse_all().to_host()
    got = pyref.concat_blocks(head + [rest])
    for k in ("label", "offset", "index", "value"):
        np.testing.assert_array_equal(got[k], cpu[k], err_msg=k)
    assert g2.tell() == g2.partition_bytes
    g2.before_first()
    assert g2.tell() == 0
