"""CPU parsers (LibSVM / LibFM / CSV) against the pure-Python grammar oracle.

Mirrors the reference's parser drivers (test/libsvm_parser_test.cc,
test/libfm_parser_test.cc, test/csv_parser_test.cc, test/strtonum_test.cc)
but with value-level assertions, plus the quirk fixes of SURVEY §7.4.
"""
import os

import numpy as np
import pytest

from dmlc_core_amd import _dmlc, data
import pyref

EDGE_LIBSVM = (
    "1 1:0.5 3:1.25e2 7\n"
    "0:2.5 qid:7 2:1 5:-3.5\r\n"
    "\n\n"
    "-1 10:1e-3 11:+4 12:.5\n"
    "   \t \n"
    "1\n"
    "0 abc 4:2 xyz:9\n"
    "2.5:3 9:1.5E+3 8:7e40 6:1.234567890123456789\n"
    "1 3:  \t 4:1\n"
    "0 1:1\n"
)


def write(path, text):
    with open(path, "w") as f:
        f.write(text)
    return path


def host_rows(path, fmt, **kw):
    uri = path + ("?" + "&".join(f"{k}={v}" for k, v in kw.items()) if kw else "")
    return pyref.concat_blocks(list(data.iter_blocks(uri, type=fmt)))


def check_libsvm(got, rows):
    assert len(got["label"]) == len(rows)
    exp_label = np.array([r[0] for r in rows], np.float32)
    np.testing.assert_array_equal(got["label"], exp_label)
    exp_w = np.array([1.0 if r[1] is None else r[1] for r in rows], np.float32)
    np.testing.assert_array_equal(got["weight"], exp_w)
    exp_qid = np.array([0 if r[2] is None else r[2] for r in rows], np.uint64)
    np.testing.assert_array_equal(got["qid"], exp_qid)
    idx = [f[0] for r in rows for f in r[3]]
    val = [1.0 if f[1] is None else f[1] for r in rows for f in r[3]]
    np.testing.assert_array_equal(got["index"], np.array(idx, np.uint64))
    np.testing.assert_array_equal(got["value"], np.array(val, np.float32))
    off = np.cumsum([0] + [len(r[3]) for r in rows]).astype(np.uint64)
    np.testing.assert_array_equal(got["offset"], off)


def test_libsvm_edge_cases(tmp_path):
    p = write(str(tmp_path / "e.libsvm"), EDGE_LIBSVM)
    check_libsvm(host_rows(p, "libsvm"), pyref.parse_libsvm(EDGE_LIBSVM))


def test_libsvm_qid_is_not_a_feature(tmp_path):
    # reference bug: qid re-parsed as a feature -> CHECK abort
    p = write(str(tmp_path / "q.libsvm"), "1 qid:3 1:1 2:2\n0 qid:4 5:1\n")
    got = host_rows(p, "libsvm")
    np.testing.assert_array_equal(got["qid"], np.array([3, 4], np.uint64))
    np.testing.assert_array_equal(got["index"], np.array([1, 2, 5], np.uint64))


def test_libsvm_partial_weights_backfilled(tmp_path):
    # reference bug: misaligned weights when only some rows have one
    p = write(str(tmp_path / "w.libsvm"), "1 1:1\n0:0.25 2:1\n1 3:1\n")
    got = host_rows(p, "libsvm")
    np.testing.assert_array_equal(got["weight"], np.array([1.0, 0.25, 1.0], np.float32))


def test_libsvm_negative_index_raises(tmp_path):
    p = write(str(tmp_path / "n.libsvm"), "1 -3:1\n")
    with pytest.raises(Exception):
        list(data.iter_blocks(p, type="libsvm"))


def test_libsvm_single_pass_token_path_matches_grammar(tmp_path):
    """Tokens at the edge of the single-pass `digits[:number]` fast path (it must
    hand every other shape to the general ParsePair grammar unchanged)."""
    text = ("1 12.5:3 5: 5:abc +3:1 1e2:3 7:1.5.3 4:-2 9:.5x 3x:2 8:1e+2 6:0.5:9 2\n"
            "0 10 11:7 12:-.25 13:+1.5e-3 4294967297:1 14:1e40\n")
    p = write(str(tmp_path / "t.libsvm"), text)
    check_libsvm(host_rows(p, "libsvm"), pyref.parse_libsvm(text))


@pytest.mark.parametrize("nthread", [1, 3, 8])
def test_libsvm_synthetic_matches_oracle(tmp_path, nthread):
    p = str(tmp_path / "s.libsvm")
    data.write_synthetic(p, 0, 3000, format="libsvm", seed=5, weight_every=7, qid=True)
    text = open(p).read()
    got = host_rows(p, "libsvm", nthread=nthread)
    check_libsvm(got, pyref.parse_libsvm(text))


@pytest.mark.parametrize("text", [
    "1 1:2:0.5 3:4 5:6:7e1 junk 2\n0:2 7:8:9\n\n1 1:1:1\n",
    # shapes at the edge of the single-pass field:index[:value] path
    "1 3:4:0.5 3:4 3:4: 3x:4:1 3:4:-1.5 3:4:1e2 +3:4:1 3:4:abc 3:4:1.5.2 3:4:2:9 12.5:3:1\n"
    "0 10:20 11:21:.25 4294967297:5:1 7:8:+2.5e-1 9:9:5.\n",
])
def test_libfm_matches_oracle(tmp_path, text):
    p = write(str(tmp_path / "f.libfm"), text)
    got = pyref.concat_blocks(list(data.iter_blocks(p, type="libfm")))
    rows = pyref.parse_libfm(text)
    np.testing.assert_array_equal(got["label"], np.array([r[0] for r in rows], np.float32))
    np.testing.assert_array_equal(got["field"], np.array([f[0] for r in rows for f in r[2]], np.uint64))
    np.testing.assert_array_equal(got["index"], np.array([f[1] for r in rows for f in r[2]], np.uint64))
    vals = [1.0 if f[2] is None else f[2] for r in rows for f in r[2]]
    np.testing.assert_array_equal(got["value"], np.array(vals, np.float32))


def test_libfm_synthetic(tmp_path):
    p = str(tmp_path / "s.libfm")
    data.write_synthetic(p, 0, 2000, format="libfm", seed=2)
    rows = pyref.parse_libfm(open(p).read())
    got = pyref.concat_blocks(list(data.iter_blocks(p, type="libfm")))
    assert len(got["label"]) == len(rows)
    np.testing.assert_array_equal(got["index"], np.array([f[1] for r in rows for f in r[2]], np.uint64))


@pytest.mark.parametrize("label_column", [-1, 0, 2])
def test_csv_matches_oracle(tmp_path, label_column):
    text = "1,2,3\n4.5,,6\n  7 ,8,9,10\r\n1e2,-2,3\n"
    p = write(str(tmp_path / "c.csv"), text)
    got = pyref.concat_blocks(list(data.iter_blocks(p + f"?label_column={label_column}", type="csv")))
    rows = pyref.parse_csv(text, label_column)
    np.testing.assert_array_equal(got["label"], np.array([r[0] for r in rows], np.float32))
    np.testing.assert_array_equal(got["value"], np.array([v for r in rows for v in r[1]], np.float32))
    idx = [i for r in rows for i in range(len(r[1]))]
    np.testing.assert_array_equal(got["index"], np.array(idx, np.uint64))


@pytest.mark.parametrize("delim", [",", ";", ":", "|", "e"])
def test_csv_junk_fields_match_oracle(tmp_path, delim):
    """Fields with bytes after the number (junk, a second number, blanks
    before the delimiter, empty fields): the direct-delimiter fast path falls
    back to the delimiter search and gives the reference's values."""
    rows_txt = ["1.5abc,2,3", "  4 ,x5,6.25e1y", "7,,8.,", "-.5,+9,1e", "12 34,5 ,6"]
    text = "\n".join(r.replace(",", delim) for r in rows_txt) + "\n"
    p = write(str(tmp_path / "j.csv"), text)
    # ('e' can be part of a number: the reference's delimiter search path)
    q = p + f"?delimiter={delim}&label_column=1"
    got = pyref.concat_blocks(list(data.iter_blocks(q, type="csv")))
    rows = pyref.parse_csv(text, 1, delim)
    np.testing.assert_array_equal(got["label"], np.array([r[0] for r in rows], np.float32))
    np.testing.assert_array_equal(got["value"], np.array([v for r in rows for v in r[1]], np.float32))
    np.testing.assert_array_equal(got["offset"], np.cumsum([0] + [len(r[1]) for r in rows]))


# trailing delimiters, derived by hand from the reference loop
# (csv_parser.h:83-96: parse, skip to ',', step over it, stop at the line end)
CSV_TRAILING = "1,2,\n3,,\n,\n4,5\n6,\n"
CSV_TRAILING_ROWS = [[1.0, 2.0], [3.0, 0.0], [0.0], [4.0, 5.0], [6.0]]


def test_csv_trailing_delimiter_matches_reference(tmp_path):
    p = write(str(tmp_path / "t.csv"), CSV_TRAILING)
    got = pyref.concat_blocks(list(data.iter_blocks(p, type="csv")))
    np.testing.assert_array_equal(got["offset"], np.cumsum([0] + [len(r) for r in CSV_TRAILING_ROWS]))
    np.testing.assert_array_equal(got["value"], np.array(sum(CSV_TRAILING_ROWS, []), np.float32))
    assert [r[1] for r in pyref.parse_csv(CSV_TRAILING)] == CSV_TRAILING_ROWS
    # label column 1 of '6,' is missing: label 0
    got = pyref.concat_blocks(list(data.iter_blocks(p + "?label_column=1", type="csv")))
    np.testing.assert_array_equal(got["label"], np.array([2, 0, 0, 5, 0], np.float32))


def test_csv_auto_format(tmp_path):
    p = write(str(tmp_path / "a.csv"), "1,2\n3,4\n")
    got = pyref.concat_blocks(list(data.iter_blocks(p + "?format=csv&label_column=0", type="auto")))
    np.testing.assert_array_equal(got["label"], np.array([1, 3], np.float32))


def test_index64_parser(tmp_path):
    p = write(str(tmp_path / "b.libsvm"), "1 4294967300:1 5:2\n")
    got = pyref.concat_blocks(list(data.iter_blocks(p, type="libsvm", index64=True)))
    np.testing.assert_array_equal(got["index"], np.array([4294967300, 5], np.uint64))


def test_strtof_matches_reference_arithmetic(tmp_path):
    vals = ["0", "1", "-1.5", "3.14159265358979", "1e10", "1e-10", "7e40", "-2.5E+3",
            "0.000001", "123456789012", ".5", "5.", "1.2.3", "1e", "9.87654321e-5"]
    text = "".join(f"{v} 1:{v}\n" for v in vals)
    p = write(str(tmp_path / "f.libsvm"), text)
    got = host_rows(p, "libsvm")
    exp = np.array([pyref.strtof(v) for v in vals], np.float32)
    np.testing.assert_array_equal(got["label"], exp)
    np.testing.assert_array_equal(got["value"], exp)


def test_rowblockiter_numcol_and_cache(tmp_path):
    p = str(tmp_path / "r.libsvm")
    data.write_synthetic(p, 0, 500, format="libsvm", seed=1, num_features=1000)
    it = data.RowBlockIter(p, type="libsvm")
    n = 0
    while it.next():
        n += len(it.value()["label"])
    assert n == 500
    assert it.num_col() <= 1000
    cache = str(tmp_path / "r.cache")
    it2 = data.RowBlockIter(p + "#" + cache, type="libsvm")
    for _ in range(2):
        it2.before_first()
        m = 0
        while it2.next():
            m += len(it2.value()["label"])
        assert m == 500
    assert it2.num_col() == it.num_col()
    assert os.path.exists(cache)
