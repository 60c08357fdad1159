"""One-pass resident CSR fill (k_tile_fill<kOnePass>: look-back instead of the
C1 count + C2 scan, written into the target's capacity, overflow -> grow ->
run again).  Every HBM-replayed epoch must equal the CPU parser bit for bit,
whatever the target (reused, fresh, too small), the data (weights first seen
late, irregular chunks, qid data -> counted path) and the chunk sizes.
(`one_pass=1`: the mode is opt-in, see DeviceParserConfig::one_pass.)"""
import numpy as np
import pytest

from dmlc_core_amd import data
import pyref

pytestmark = pytest.mark.gpu


def cpu_rows(uri, fmt):
    return pyref.concat_blocks(list(data.iter_blocks(uri, 0, 1, type=fmt)))


def assert_same(a, b, field=False):
    for k in ("label", "weight", "qid", "offset", "index", "value"):
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)
    if field:
        np.testing.assert_array_equal(a["field"], b["field"])


def replay(gp, csr=None):
    gp.before_first()
    if csr is None:
        csr = data.DeviceCSR()
    else:
        csr.clear()
    gp.parse_all(csr)
    return csr


@pytest.mark.parametrize("fmt", ["libsvm", "libfm"])
@pytest.mark.parametrize("replay_mb", [0.0625, 1])
def test_one_pass_replay_equals_cpu(tmp_path, fmt, replay_mb):
    """streaming epoch 1 (counted), then replays in one pass into the reused
    target, into a fresh one (capacity 0: the first chunk overflows, the
    target is sized for the partition and the chunk runs again) and into the
    reused one again; weights appear only in the last file"""
    d = tmp_path / "c"
    d.mkdir()
    for i in range(3):
        data.write_synthetic(str(d / f"p{i}.{fmt}"), i * 2000, (i + 1) * 2000, format=fmt,
                             seed=41, weight_every=3 if i == 2 else 0)
    c = cpu_rows(str(d), fmt)
    gp = data.GPUParser(str(d), format=fmt, chunk_bytes=48 * 1024, hbm_cache=1,
                        replay_chunk_mb=replay_mb, one_pass=1)
    csr = data.DeviceCSR()
    csr = replay(gp, csr)  # epoch 1: streams, fills the HBM cache
    assert_same(pyref.concat_blocks([csr.to_host()]), c, field=fmt == "libfm")
    assert gp.stats()["one_pass_chunks"] == 0
    for target in (csr, None, csr):
        out = replay(gp, target)
        assert_same(pyref.concat_blocks([out.to_host()]), c, field=fmt == "libfm")
        assert out.max_index == csr.max_index
    st = gp.stats()
    assert st["one_pass_chunks"] >= 3
    assert st["one_pass_reruns"] >= 1  # the fresh target: overflow (and the weight column)
    assert st["exact_chunks"] == 0


def test_one_pass_irregular_chunk_takes_the_exact_kernels(tmp_path):
    """a blank-started line, a stray control byte and a junk token -- each
    flagged by the one-pass kernel itself -- send their chunk to the exact
    kernels; the other chunks stay one-pass"""
    d = tmp_path / "c"
    d.mkdir()
    for i in range(4):
        data.write_synthetic(str(d / f"p{i}.libsvm"), i * 1500, (i + 1) * 1500, seed=43)
    with open(d / "p1.libsvm", "a") as f:
        f.write(" 1 3:1\n")
    with open(d / "p2.libsvm", "a") as f:
        f.write("1 3:1\x0b 4:1\n")
    with open(d / "p3.libsvm", "a") as f:
        f.write("1 junk 4:1\n")
    c = cpu_rows(str(d), "libsvm")
    gp = data.GPUParser(str(d), chunk_bytes=32 * 1024, hbm_cache=1, replay_chunk_mb=0.0625,
                        one_pass=1)
    csr = data.DeviceCSR()
    done = []
    for _ in range(3):
        csr = replay(gp, csr)
        assert_same(pyref.concat_blocks([csr.to_host()]), c)
        done.append(gp.stats()["one_pass_chunks"])
    # junk is no qid data: the regular chunks stay one-pass in every replay
    assert 0 < done[1] < done[2]
    assert gp.stats()["exact_chunks"] > 0


def test_one_pass_qid_data_takes_the_counted_path(tmp_path):
    """`qid:` tokens: the one-pass kernel flags them (it has no zeroed qid
    column to write into); the chunk and every later one take the counted
    tile path, with equal output"""
    p = str(tmp_path / "q.libsvm")
    data.write_synthetic(p, 0, 6000, format="libsvm", seed=47, weight_every=4, qid=True)
    c = cpu_rows(p, "libsvm")
    gp = data.GPUParser(p, chunk_bytes=64 * 1024, hbm_cache=1, one_pass=1)
    csr = data.DeviceCSR()
    for _ in range(3):
        csr = replay(gp, csr)
        assert_same(pyref.concat_blocks([csr.to_host()]), c)
    assert gp.stats()["one_pass_chunks"] == 0
    assert gp.stats()["exact_chunks"] == 0


def test_one_pass_token_edges_and_shapes(tmp_path):
    """tokens of every length straddling tiles / LDS halos / windows, the
    last line without EOL, and the skewed / mixed synthetic shapes (lines
    longer than a tile, exponents, valueless features): replays equal CPU"""
    rng = np.random.default_rng(5)
    lines = []
    for r in range(2500):
        toks = []
        for _ in range(int(rng.integers(1, 12))):
            digits = "".join(str(int(x)) for x in rng.integers(0, 10, int(rng.integers(1, 70))))
            toks.append(f"{int(rng.integers(0, 1 << 20))}:0.{digits}")
        lines.append(f"{r % 3} " + " ".join(toks))
    p = str(tmp_path / "edge.libsvm")
    with open(p, "w") as f:
        f.write("\n".join(lines))
    for path in (p,):
        c = cpu_rows(path, "libsvm")
        gp = data.GPUParser(path, chunk_bytes=40 * 1024, hbm_cache=1, one_pass=1)
        csr = data.DeviceCSR()
        for _ in range(2):
            csr = replay(gp, csr)
            assert_same(pyref.concat_blocks([csr.to_host()]), c)
        assert gp.stats()["one_pass_chunks"] > 0
    q = str(tmp_path / "skew.libsvm")
    data.write_synthetic(q, 0, 20000, format="libsvm", seed=9, shape="skewed")
    c = cpu_rows(q, "libsvm")
    gp = data.GPUParser(q, chunk_bytes=256 * 1024, hbm_cache=1, one_pass=1)
    csr = data.DeviceCSR()
    for _ in range(2):
        csr = replay(gp, csr)
        assert_same(pyref.concat_blocks([csr.to_host()]), c)
    assert gp.stats()["one_pass_chunks"] > 0


def test_one_pass_streaming_next_is_unchanged(tmp_path):
    """Next() (one block per chunk, a fresh block each time) keeps the counted
    path; only ParseAll over resident text runs one pass"""
    p = str(tmp_path / "s.libsvm")
    data.write_synthetic(p, 0, 5000, format="libsvm", seed=51)
    c = cpu_rows(p, "libsvm")
    gp = data.GPUParser(p, chunk_bytes=64 * 1024, hbm_cache=1, one_pass=1)
    replay(gp)
    gp.before_first()
    blocks = []
    while gp.next():
        blocks.append(gp.value_to_host())
    assert_same(pyref.concat_blocks(blocks), c)
    assert gp.stats()["one_pass_chunks"] == 0
