"""GPU ingestion (HIP kernels K1-K4/K8 + pinned ring) vs the CPU parsers:
bit-identical CSR, compared row by row on concatenated blocks (block
boundaries differ by design).  Chunk sizes are forced small so that records
straddle chunk, file and shard boundaries."""
import os

import numpy as np
import pytest

from dmlc_core_amd import data
import pyref

pytestmark = pytest.mark.gpu


def gpu_rows(uri, fmt, nparts=1, index64=False, **cfg):
    parts = []
    for r in range(nparts):
        csr = data.GPUParser(uri, r, nparts, format=fmt, index64=index64, **cfg).parse_all()
        h = csr.to_host()
        parts.append(h)
    return pyref.concat_blocks(parts)


def cpu_rows(uri, fmt, nparts=1, index64=False):
    blocks = []
    for r in range(nparts):
        blocks.extend(data.iter_blocks(uri, r, nparts, type=fmt, index64=index64))
    return pyref.concat_blocks(blocks)


def assert_same(a, b, field=False):
    for k in ("label", "weight", "qid", "offset", "index", "value"):
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)
    if field:
        np.testing.assert_array_equal(a["field"], b["field"])


@pytest.mark.parametrize("chunk_kb", [4, 64, 4096])
def test_libsvm_gpu_equals_cpu(tmp_path, chunk_kb):
    p = str(tmp_path / "s.libsvm")
    data.write_synthetic(p, 0, 4000, format="libsvm", seed=11, weight_every=5, qid=True)
    g = gpu_rows(p, "libsvm", chunk_bytes=chunk_kb * 1024, read_threads=3)
    c = cpu_rows(p, "libsvm")
    assert_same(g, c)


@pytest.mark.parametrize("fast", [0, 1])
@pytest.mark.parametrize("weights", [0, 3])
def test_fast_and_exact_paths_agree(tmp_path, fast, weights):
    p = str(tmp_path / "s.libsvm")
    data.write_synthetic(p, 0, 3000, format="libsvm", seed=21, weight_every=weights)
    g = gpu_rows(p, "libsvm", chunk_bytes=64 * 1024, fast_path=fast)
    assert_same(g, cpu_rows(p, "libsvm"))


@pytest.mark.parametrize("zero_copy", [0, 1])
def test_zero_copy_and_pinned_ring_agree(tmp_path, zero_copy):
    d = tmp_path / "zc"
    d.mkdir()
    for i in range(3):
        data.write_synthetic(str(d / f"p{i}.libsvm"), i * 900, (i + 1) * 900, seed=13)
    with open(d / "p9.libsvm", "w") as f:
        f.write("1 1:1 2:2\n0 3:3")  # no trailing newline at a file boundary
    for nparts in (1, 3):
        g = gpu_rows(str(d), "libsvm", nparts=nparts, chunk_bytes=48 * 1024, zero_copy=zero_copy)
        assert_same(g, cpu_rows(str(d), "libsvm", nparts=nparts))
    gp = data.GPUParser(str(d), chunk_bytes=48 * 1024, zero_copy=zero_copy)
    gp.parse_all()
    assert gp.stats()["zero_copy"] == bool(zero_copy)


@pytest.mark.parametrize("fmt,junk", [("libsvm", "1 qid:9 1:1 2:2\n0 junk 3:1\n"),
                                      ("libfm", "1 x:1:1 2:2:2\n0 #c 3:3:1\n")])
def test_irregular_chunks_fall_back(tmp_path, fmt, junk):
    # qid tokens and digit-less tokens are not handled by the token-parallel
    # path (the fill flags them on its fallback decode): those chunks must be
    # re-parsed exactly, the rest stay fast
    p = str(tmp_path / f"m.{fmt}")
    data.write_synthetic(p, 0, 2000, format=fmt, seed=5)
    with open(p, "a") as f:
        f.write(junk)
    data.write_synthetic(str(tmp_path / "tail"), 2000, 4000, format=fmt, seed=5)
    with open(p, "a") as f:
        f.write(open(str(tmp_path / "tail")).read())
    gp = data.GPUParser(p, format=fmt, chunk_bytes=64 * 1024)
    csr = gp.parse_all()
    st = gp.stats()
    assert 0 < st["exact_chunks"] < st["chunks"]
    assert_same(pyref.concat_blocks([csr.to_host()]), cpu_rows(p, fmt), field=fmt == "libfm")


def test_libsvm_gpu_edge_cases(tmp_path):
    from test_cpu_parsers import EDGE_LIBSVM
    p = str(tmp_path / "e.libsvm")
    with open(p, "w") as f:
        f.write(EDGE_LIBSVM * 50)
    assert_same(gpu_rows(p, "libsvm", chunk_bytes=4096), cpu_rows(p, "libsvm"))


def test_long_lines_cross_lds_window(tmp_path):
    # lines of ~20 KB (far beyond the 2 KiB per-wave LDS window) and long tokens
    rng = np.random.default_rng(0)
    lines = []
    for r in range(40):
        n = int(rng.integers(500, 1500))
        idx = np.sort(rng.integers(0, 1 << 30, n))
        toks = " ".join(f"{i}:{rng.random():.9f}" for i in idx)
        lines.append(f"{r % 2} {toks} 7:{'1' * 300}.5")
    p = str(tmp_path / "long.libsvm")
    with open(p, "w") as f:
        f.write("\n".join(lines) + "\n")
    assert_same(gpu_rows(p, "libsvm", chunk_bytes=128 * 1024), cpu_rows(p, "libsvm"))


@pytest.mark.parametrize("nparts", [1, 2, 3, 8])
def test_sharded_multifile_union(tmp_path, nparts):
    d = tmp_path / "parts"
    d.mkdir()
    for i in range(4):
        data.write_synthetic(str(d / f"part-{i}.libsvm"), i * 700, (i + 1) * 700, seed=4)
    # a file without trailing newline: the split inserts one between files
    with open(d / "part-9.libsvm", "w") as f:
        f.write("1 1:1 2:2\n0 3:3")
    g = gpu_rows(str(d), "libsvm", nparts=nparts, chunk_bytes=32 * 1024)
    c = cpu_rows(str(d), "libsvm", nparts=nparts)
    assert_same(g, c)
    assert len(g["label"]) == 2802


def test_libfm_gpu_equals_cpu(tmp_path):
    p = str(tmp_path / "s.libfm")
    data.write_synthetic(p, 0, 3000, format="libfm", seed=3)
    with open(p, "a") as f:
        f.write("1 1:2:0.5 3:4 5:6:7e1 junk 2\n0:2 7:8:9\n")
    g = gpu_rows(p, "libfm", chunk_bytes=64 * 1024)
    c = cpu_rows(p, "libfm")
    assert_same(g, c, field=True)


@pytest.mark.parametrize("fast_path", [1, 0])
@pytest.mark.parametrize("label_column", [-1, 1])
def test_csv_trailing_delimiter_matches_reference(tmp_path, fast_path, label_column):
    """a line ending in the delimiter has no empty last field (reference
    csv_parser.h:83-96), on the tile path and on the exact per-line kernels"""
    from test_cpu_parsers import CSV_TRAILING, CSV_TRAILING_ROWS
    p = str(tmp_path / "t.csv")
    with open(p, "w") as f:
        f.write(CSV_TRAILING * 50)
    rows = CSV_TRAILING_ROWS * 50
    g = gpu_rows(p, "csv", label_column=label_column, fast_path=fast_path)
    if label_column < 0:
        np.testing.assert_array_equal(g["offset"], np.cumsum([0] + [len(r) for r in rows]))
        np.testing.assert_array_equal(g["value"], np.array(sum(rows, []), np.float32))
    else:
        lab = [r[1] if len(r) > 1 else 0.0 for r in rows]
        np.testing.assert_array_equal(g["label"], np.array(lab, np.float32))
    assert_same(g, cpu_rows(p + f"?label_column={label_column}", "csv"))


@pytest.mark.parametrize("label_column", [-1, 0, 3])
def test_csv_gpu_equals_cpu(tmp_path, label_column):
    p = str(tmp_path / "s.csv")
    data.write_synthetic(p, 0, 3000, format="csv", seed=8)
    with open(p, "a") as f:
        f.write("1,,3\n  7 ,8,9,10\r\n")
    uri = p + f"?label_column={label_column}"
    g = gpu_rows(uri, "csv", chunk_bytes=64 * 1024, label_column=label_column)
    c = cpu_rows(uri, "csv")
    np.testing.assert_array_equal(g["label"], c["label"])
    np.testing.assert_array_equal(g["offset"], c["offset"])
    np.testing.assert_array_equal(g["index"], c["index"])
    np.testing.assert_array_equal(g["value"], c["value"])


CSV_FIELDS = ["1", "0.5", "-2", "+3.75", ".25", "5.", "", " 7", "  -1.5", "1e3", "2.5E-2",
              "1.5.3", "3x", "123456789.5", "-", "+.5", "12345678", "1234567", "0.1234567",
              "9.87654321", "x", "4 ", "\t8"]


@pytest.mark.parametrize("delim", [",", "\t"])
@pytest.mark.parametrize("label_column,weight_column", [(-1, -1), (0, -1), (2, 0), (1, 3), (0, 5)])
def test_csv_shape_fuzz_matches_cpu(tmp_path, delim, label_column, weight_column):
    """CSV tile path (lane per row) vs the CPU parser: every field shape the
    register-window decoder takes and many it hands to StrToFloat (blanks,
    junk, exponents, long digit runs, empty fields), short rows that lack the
    label / weight column, CRLF, blank lines, no final newline; plus rows over
    the 4 KiB tile extension, which send their chunk to the exact kernels."""
    rng = np.random.default_rng(40 + label_column * 7 + weight_column)
    fields = [f for f in CSV_FIELDS if delim not in f]
    lines = []
    for r in range(4000):
        n = int(rng.integers(1, 40))
        lines.append(delim.join(fields[int(rng.integers(len(fields)))] for _ in range(n)))
        if rng.random() < 0.02:
            lines.append("")
    p = str(tmp_path / "f.csv")
    with open(p, "w", newline="") as f:
        f.write("\r\n".join(lines[:100]) + "\n" + "\n".join(lines[100:]))
    q = f"?label_column={label_column}&weight_column={weight_column}"
    if delim != ",":
        q += "&delimiter=\t"
    cfg = dict(label_column=label_column, weight_column=weight_column, delimiter=delim)
    c = cpu_rows(p + q, "csv")
    for chunk in (8192, 64 * 1024, 1 << 20):
        gp = data.GPUParser(p + q, format="csv", chunk_bytes=chunk, **cfg)
        g = pyref.concat_blocks([gp.parse_all().to_host()])
        for k in ("label", "weight", "offset", "index", "value"):
            np.testing.assert_array_equal(g[k], c[k], err_msg=f"{k} chunk={chunk}")
        assert gp.stats()["exact_chunks"] == 0
    # wide rows (> 4 KiB past their tile): exact kernels for those chunks
    wide = str(tmp_path / "wide.csv")
    with open(wide, "w") as f:
        f.write("\n".join(lines[:500]) + "\n")
        f.write(delim.join(["1.25"] * 3000) + "\n")
        f.write("\n".join(lines[500:1500]))
    gp = data.GPUParser(wide + q, format="csv", chunk_bytes=32 * 1024, **cfg)
    g = pyref.concat_blocks([gp.parse_all().to_host()])
    c = cpu_rows(wide + q, "csv")
    for k in ("label", "weight", "offset", "index", "value"):
        np.testing.assert_array_equal(g[k], c[k], err_msg=k)
    st = gp.stats()
    assert 0 < st["exact_chunks"] < st["chunks"]


def test_index64_gpu(tmp_path):
    p = str(tmp_path / "b.libsvm")
    with open(p, "w") as f:
        f.write("1 4294967300:1 5:2\n0 18446744073709551615:3\n")
    g = gpu_rows(p, "libsvm", index64=True)
    c = cpu_rows(p, "libsvm", index64=True)
    assert_same(g, c)


def test_streaming_next_blocks(tmp_path):
    p = str(tmp_path / "s.libsvm")
    data.write_synthetic(p, 0, 5000, seed=2)
    gp = data.GPUParser(p, chunk_bytes=256 * 1024)
    for _epoch in range(2):
        blocks = []
        while gp.next():
            blocks.append(gp.value_to_host())
        assert len(blocks) > 3
        assert_same(pyref.concat_blocks(blocks), cpu_rows(p, "libsvm"))
        gp.before_first()


def test_resident_parse_repeat_and_torch(tmp_path):
    import torch
    p = str(tmp_path / "s.libsvm")
    data.write_synthetic(p, 0, 3000, seed=9)
    gp = data.GPUParser(p, chunk_bytes=100 * 1024)
    csr = data.DeviceCSR()
    for _ in range(3):
        gp.before_first()
        csr.clear()
        gp.parse_all(csr)
        assert csr.rows == 3000
    t = data.csr_to_torch(csr)
    assert t["index"].device.type == "cuda"
    c = cpu_rows(p, "libsvm")
    np.testing.assert_array_equal(t["label"].cpu().numpy(), c["label"])
    off = t["offset"].cpu()
    off = (off.view(torch.int64) if off.dtype != torch.int64 else off).numpy()
    np.testing.assert_array_equal(off.astype(np.uint64), c["offset"])


def test_negative_index_raises_on_gpu(tmp_path):
    p = str(tmp_path / "n.libsvm")
    with open(p, "w") as f:
        f.write("1 -3:1\n")
    with pytest.raises(Exception):
        data.GPUParser(p).parse_all()


@pytest.mark.parametrize("zero_copy", [0, 1])
def test_hbm_epoch_cache_replay_and_resume(tmp_path, zero_copy):
    """hbm_cache=1: epoch 1 streams and keeps the text in HBM; later epochs
    (parse_all and streaming next) replay from HBM with identical output, and a
    resume cursor that is a chunk boundary replays from there."""
    d = tmp_path / "c"
    d.mkdir()
    for i in range(3):
        data.write_synthetic(str(d / f"p{i}.libsvm"), i * 1500, (i + 1) * 1500, seed=31,
                             weight_every=4 if i == 2 else 0)
    c = cpu_rows(str(d), "libsvm")
    gp = data.GPUParser(str(d), chunk_bytes=64 * 1024, zero_copy=zero_copy, hbm_cache=1)
    csr = data.DeviceCSR()
    for _ in range(3):
        gp.before_first()
        csr.clear()
        gp.parse_all(csr)
        assert_same(pyref.concat_blocks([csr.to_host()]), c)
    gp.before_first()
    head = [gp.value_to_host() for _ in range(2) if gp.next()]
    cursor = gp.tell()
    assert 0 < cursor < gp.partition_bytes
    rest = []
    while gp.next():
        rest.append(gp.value_to_host())
    assert_same(pyref.concat_blocks(head + rest), c)
    gp.seek(cursor)
    again = []
    while gp.next():
        again.append(gp.value_to_host())
    assert_same(pyref.concat_blocks(head + again), c)


@pytest.mark.parametrize("replay_mb", [0.0625, 0.25])
def test_hbm_replay_prelaunched_counts(tmp_path, replay_mb):
    """Replayed ParseAll queues the next resident chunk's count + scan behind
    the current fill (a second scratch set).  Many merged chunks, a weight
    column first seen late (the fill re-runs its chunk), an irregular chunk
    in the middle (exact fallback) and a resume in between: every epoch equals
    the CPU parser."""
    d = tmp_path / "c"
    d.mkdir()
    for i in range(3):
        data.write_synthetic(str(d / f"p{i}.libsvm"), i * 1500, (i + 1) * 1500, seed=37,
                             weight_every=5 if i == 2 else 0)
    with open(d / "p1.libsvm", "a") as f:
        f.write("1 junk 4:1\n")  # a token the tile path leaves to the exact kernels
    c = cpu_rows(str(d), "libsvm")
    gp = data.GPUParser(str(d), chunk_bytes=32 * 1024, hbm_cache=1, replay_chunk_mb=replay_mb)
    csr = data.DeviceCSR()
    for epoch in range(3):
        gp.before_first()
        csr.clear()
        gp.parse_all(csr)
        assert_same(pyref.concat_blocks([csr.to_host()]), c)
        if epoch == 1:
            gp.before_first()
            assert gp.next()  # a partial streaming pass between two replays
    assert gp.stats()["exact_chunks"] > 0


def test_weight_column_first_seen_in_a_late_chunk(tmp_path):
    """The tile fill learns about weights only when it meets one: the column
    is allocated then (earlier rows 1.0) and that chunk is written again."""
    p = str(tmp_path / "w.libsvm")
    data.write_synthetic(p, 0, 3000, seed=17)
    with open(p, "a") as f:
        f.write("1:0.25 4:1 9:2\n0 3:1\n1:3.5 1:1\n")
    g = gpu_rows(p, "libsvm", chunk_bytes=32 * 1024)
    c = cpu_rows(p, "libsvm")
    assert_same(g, c)
    assert c["weight"][-3] == np.float32(0.25) and c["weight"][0] == 1.0


def test_tokens_at_tile_and_window_edges(tmp_path):
    """Tokens of every length 1..70 placed so they straddle the 8 KiB tile, the
    64 B LDS halo and the 32 B parse window; the last line has no newline."""
    rng = np.random.default_rng(3)
    lines = []
    for r in range(3000):
        n = int(rng.integers(1, 12))
        toks = []
        for _ in range(n):
            L = int(rng.integers(1, 70))
            digits = "".join(str(int(x)) for x in rng.integers(0, 10, L))
            toks.append(f"{int(rng.integers(0, 1 << 20))}:0.{digits}")
        lines.append(f"{r % 3} " + " ".join(toks))
    p = str(tmp_path / "edge.libsvm")
    with open(p, "w") as f:
        f.write("\n".join(lines))
    for chunk in (8192, 40 * 1024, 1 << 20):
        assert_same(gpu_rows(p, "libsvm", chunk_bytes=chunk), cpu_rows(p, "libsvm"))


def test_token_shape_fuzz_matches_cpu(tmp_path):
    """Labels / features in every shape the single-pass SWAR path accepts and
    many it must hand to the generic grammar (signs, exponents, second dots,
    junk bytes, empty values, long digit runs, weights)."""
    rng = np.random.default_rng(12)
    labels = ["1", "0", "-1", "+1", "0.5", "-0", "3.25", ".5", "1:0.25", "-1:2", "2:-0.5",
              "1e2", "12345678", "1.5e-1:3", "7:", "1:2:3"]
    values = ["1", "0.5", "-2", "+3.75", ".25", "5.", "", "1e3", "2.5E-2", "1.5.3", "3x",
              "123456789.5", "0.000000000000000000000001", "-.5", "7:9", "12345678", "1234567"]
    lines = []
    for r in range(6000):
        toks = [labels[int(rng.integers(len(labels)))]]
        for _ in range(int(rng.integers(0, 9))):
            idx = str(int(rng.integers(0, 1 << 31)))
            if rng.random() < 0.1:
                toks.append(idx)
            else:
                toks.append(idx + ":" + values[int(rng.integers(len(values)))])
        lines.append(" ".join(toks))
    p = str(tmp_path / "fuzz.libsvm")
    with open(p, "w") as f:
        f.write("\n".join(lines) + "\n")
    for chunk in (16 * 1024, 1 << 20):
        assert_same(gpu_rows(p, "libsvm", chunk_bytes=chunk), cpu_rows(p, "libsvm"))
    # the same for LibFM triples
    fm = []
    for r in range(3000):
        toks = [labels[int(rng.integers(len(labels)))]]
        for _ in range(int(rng.integers(1, 7))):
            t = f"{int(rng.integers(0, 50))}:{int(rng.integers(0, 1 << 20))}"
            if rng.random() < 0.85:
                t += ":" + values[int(rng.integers(len(values)))]
            toks.append(t)
        fm.append(" ".join(toks))
    q = str(tmp_path / "fuzz.libfm")
    with open(q, "w") as f:
        f.write("\n".join(fm) + "\n")
    assert_same(gpu_rows(q, "libfm", chunk_bytes=16 * 1024), cpu_rows(q, "libfm"), field=True)


@pytest.mark.parametrize("hbm_cache", [0, 1])
def test_zero_copy_windowed_pinning(tmp_path, hbm_cache):
    """A partition above the pin budget is mapped + registered in sliding
    windows (background prefetch, at most two pinned); output unchanged."""
    d = tmp_path / "w"
    d.mkdir()
    for i in range(3):
        data.write_synthetic(str(d / f"p{i}.libsvm"), i * 4000, (i + 1) * 4000, seed=19)
    c = cpu_rows(str(d), "libsvm")
    g = data.GPUParser(str(d), chunk_bytes=96 * 1024, zero_copy=1, zc_pin_budget_mb=1,
                       zc_window_mb=0.5, hbm_cache=hbm_cache)
    for _ in range(2):
        g.before_first()
        assert_same(pyref.concat_blocks([g.parse_all().to_host()]), c)
    assert g.stats()["zero_copy"]
    g.before_first()
    blocks = []
    while g.next():
        blocks.append(g.value_to_host())
    assert_same(pyref.concat_blocks(blocks), c)


def test_two_level_scan_and_finish_on_large_chunks(tmp_path):
    """Chunks above 8192 tiles (64 MiB) take the multi-workgroup tile scan and
    finish fold: one 192 MiB chunk, and HBM-cache replay passes merged up to
    1 GiB, must equal the CPU parser; the fused hashed batch of one big chunk
    must equal the one built from 4 MiB chunks."""
    p = str(tmp_path / "big.libsvm")
    data.write_synthetic(p, 0, 250_000, format="libsvm", seed=5)
    assert os.path.getsize(p) > 100 << 20
    c = cpu_rows(p, "libsvm")
    assert_same(gpu_rows(p, "libsvm", chunk_bytes=192 << 20), c)
    gp = data.GPUParser(p, format="libsvm", chunk_bytes=16 << 20, hbm_cache=1)
    for _ in range(2):  # epoch 1 streams 16 MiB chunks, epoch 2 replays one merged pass
        gp.before_first()
        csr = data.DeviceCSR()
        gp.parse_all(csr)
        assert_same(pyref.concat_blocks([csr.to_host()]), c)
    # f32 rows (LDS accumulation order may differ between runs in the last bit)
    big = data.GPUParser(p, format="libsvm", chunk_bytes=192 << 20).parse_all_hashed(
        256, seed=1, fp8=False, strategy="fused")
    small = data.GPUParser(p, format="libsvm", chunk_bytes=4 << 20).parse_all_hashed(
        256, seed=1, fp8=False, strategy="fused")
    np.testing.assert_allclose(big["x"].cpu().numpy(), small["x"].cpu().numpy(), rtol=1e-6, atol=1e-6)
    np.testing.assert_array_equal(big["label"].cpu().numpy(), c["label"])


def test_replay_chunk_limit_is_enforced(tmp_path):
    """Merged HBM-replay chunks must stay below the 32-bit offsets of the tile
    scan and the exact path's line starts: an over-large replay_chunk_mb is
    rejected up front, for text and for RecordIO."""
    from dmlc_core_amd import io
    p = str(tmp_path / "s.libsvm")
    data.write_synthetic(p, 0, 100, seed=1)
    with pytest.raises(Exception, match="replay_chunk_bytes"):
        data.GPUParser(p, hbm_cache=1, replay_chunk_mb=4096)
    r = str(tmp_path / "s.rec")
    w = io.RecordIOWriter(r)
    w.write(b"abc")
    w.close()
    with pytest.raises(Exception, match="replay_chunk_bytes"):
        io.GPURecordIO(r, hbm_cache=1, replay_chunk_mb=8192)


@pytest.mark.parametrize("nparts,zero_copy,hbm", [(1, "auto", 0), (2, "auto", 0), (2, "0", 0),
                                                   (2, "auto", 1), (1, "0", 1)])
def test_shuffled_gpu_parser_follows_input_split_shuffle(tmp_path, nparts, zero_copy, hbm):
    """ShuffledGPUParser visits the sub-shards in InputSplitShuffle's per-epoch
    order: each epoch's CSR (parse_all and streaming next) equals the CPU
    parser's rows of the sub-shards in that order -- on the zero-copy and the
    pinned-ring readers, and replayed from the HBM cache in each new order."""
    from dmlc_core_amd import _dmlc
    d = tmp_path / "s"
    d.mkdir()
    for i in range(3):
        data.write_synthetic(str(d / f"p{i}.libsvm"), i * 1500, (i + 1) * 1500, seed=23)
    with open(str(d / "p1.libsvm"), "ab") as f:  # a file whose last line has no EOL
        f.write(b"1 3:0.5 9:1")
    uri, k, seed = str(d), 4, 9
    for part in range(nparts):
        sp = data.ShuffledGPUParser(uri, part, nparts, num_shuffle_parts=k, shuffle_seed=seed,
                                    chunk_bytes=64 * 1024, zero_copy=zero_copy, hbm_cache=hbm)
        orders = []
        for epoch in range(4 if hbm else 3):
            if epoch:
                sp.before_first()
            order = list(_dmlc.shuffle_parts_order(part, nparts, k, seed, epoch))
            assert sp.order == order
            orders.append(order)
            want = cpu_rows_parts(uri, [part * k + s for s in order], nparts * k)
            if epoch < 2 or (hbm and epoch == 3):
                got = pyref.concat_blocks([sp.parse_all().to_host()])
            else:
                blocks = []
                while sp.next():
                    blocks.append(sp.value_to_host())
                got = pyref.concat_blocks(blocks)
            assert_same(got, want)
        assert len({tuple(o) for o in orders}) > 1  # the order changes between epochs
        if hbm:
            assert sp.stats()["chunks"] > 0


def cpu_rows_parts(uri, parts, nparts):
    blocks = []
    for p in parts:
        blocks.extend(data.iter_blocks(uri, p, nparts, type="libsvm"))
    return pyref.concat_blocks(blocks)


def test_shuffled_gpu_parser_resume_mid_epoch(tmp_path):
    """state_dict = (epoch, cursor): a new parser restores the epoch's visiting
    order and continues at the cursor; the rest of the epoch equals the CPU
    rows after the delivered ones.  Also reachable as ?shuffle_parts=&shuffle_seed=."""
    p = str(tmp_path / "r.libsvm")
    data.write_synthetic(p, 0, 6000, seed=31)
    k, seed = 5, 3
    sp = data.ShuffledGPUParser(p, 0, 1, num_shuffle_parts=k, shuffle_seed=seed,
                                chunk_bytes=32 * 1024)
    sp.before_first()
    sp.before_first()  # epoch 2
    want = cpu_rows_parts(p, sp.order, k)
    head = []
    for _ in range(3):
        assert sp.next()
        head.append(sp.value_to_host())
    state = sp.state_dict()
    assert state["epoch"] == 2
    sp2 = data.ShuffledGPUParser(p, 0, 1, num_shuffle_parts=k, shuffle_seed=seed,
                                 chunk_bytes=32 * 1024)
    sp2.load_state_dict(state)
    assert sp2.order == sp.order
    tail = []
    while sp2.next():
        tail.append(sp2.value_to_host())
    assert_same(pyref.concat_blocks(head + tail), want)
    g = data.GPUParser(p + f"?shuffle_parts={k}&shuffle_seed={seed}", chunk_bytes=32 * 1024)
    assert_same(pyref.concat_blocks([g.parse_all().to_host()]),
                cpu_rows_parts(p, g._p.visit_order(), k))


@pytest.mark.parametrize("fmt", ["libsvm", "libfm"])
@pytest.mark.parametrize("shape", ["skewed", "mixed"])
def test_realistic_shapes_stay_on_the_tile_path(tmp_path, fmt, shape):
    """power-law lines (some > 8 KiB), exponent / 9-12-digit / integer /
    valueless values, weights and LibSVM `qid:` tokens: the tile fast path
    takes every chunk (qid tokens are decoded beside the token list; odd
    numbers by the generic strtonum path on their lane) and equals the CPU
    parser bit for bit"""
    p = str(tmp_path / f"m.{fmt}")
    data.write_synthetic(p, 0, 30000, format=fmt, seed=13, shape=shape)
    g = data.GPUParser(p, format=fmt, chunk_bytes=256 * 1024)
    got = pyref.concat_blocks([g.parse_all().to_host()])
    assert g.stats()["exact_chunks"] == 0
    assert_same(got, cpu_rows(p, fmt), field=fmt == "libfm")


def test_qid_tokens_on_the_tile_path(tmp_path):
    """qid on every line (LETOR style), on some lines, negative and huge
    values, and tokens that only look like qid (not the second token, junk
    after the digits, a line starting with q): valid ones stay on the tile
    path, the rest send their chunk to the exact kernels; all equal the CPU"""
    p = str(tmp_path / "q.libsvm")
    data.write_synthetic(p, 0, 3000, format="libsvm", seed=2, qid=True, weight_every=3)
    g = data.GPUParser(p, chunk_bytes=64 * 1024)
    assert_same(pyref.concat_blocks([g.parse_all().to_host()]), cpu_rows(p, "libsvm"))
    assert g.stats()["exact_chunks"] == 0
    odd = str(tmp_path / "o.libsvm")
    with open(odd, "w") as f:
        f.write("1 qid:-5 3:1\n0 qid:18446744073709551615 4:2\n1 qid:7 qid:8 5:1\n")
        f.write("0 2:1 qid:9\n1 qid:3x 6:1\nqid:4 1 2:2\n1 qid: 7:1\n")
    gg = data.GPUParser(odd)
    assert_same(pyref.concat_blocks([gg.parse_all().to_host()]), cpu_rows(odd, "libsvm"))


def test_extended_number_decoder_edge_values(tmp_path):
    """the lane decoder for exponents and long fractions (token_decode.h
    parse_num_ext) against the CPU strtonum grammar: exponent clamp at 38,
    upper-case E, explicit signs, denormal results, empty exponents, 8-16
    fraction digits, and shapes it declines (8+ integer digits, 16+ fraction
    digits) that the generic path takes"""
    vals = ["1e38", "1e39", "1.5E+2", "-2.5e-40", "3e0", ".5e1", "5.e2", "1e", "2e+", "7e-",
            "0.1234567890123", "0.123456789012345", "0.1234567890123456", "12345678.5",
            "1234567.25e-3", "9.999999e-1", "+4.25e1", "-0.0e5", "6e07", "1.1e-45", "3.4e38"]
    p = str(tmp_path / "e.libsvm")
    with open(p, "w") as f:
        for r in range(400):
            v = vals[r % len(vals)]
            lab = vals[(r * 7) % len(vals)] if r % 3 == 0 else str(r % 2)
            f.write(f"{lab} {r % 50}:{v} {100 + r}:{vals[(r + 5) % len(vals)]} 7\n")
    g = data.GPUParser(p, chunk_bytes=4096)
    assert_same(pyref.concat_blocks([g.parse_all().to_host()]), cpu_rows(p, "libsvm"))
    assert g.stats()["exact_chunks"] == 0
