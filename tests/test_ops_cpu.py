"""The transpose's interleaved (index, value) pair layout as ops sees it,
checked on CPU tensors: which dicts the SpMV takes as pairs and which ones
the contiguity check rejects (the kernels themselves run in test_gpu_ops.py)."""
import pytest
import torch

from dmlc_core_amd import ops


def _pair_dict(nnz=37):
    pairs = torch.zeros((nnz, 2), dtype=torch.int32)
    pairs[:, 0] = torch.arange(nnz, dtype=torch.int32)
    pairs.view(torch.float32)[:, 1] = torch.linspace(-1, 1, nnz)
    return {"offset": torch.tensor([0, nnz], dtype=torch.int64), "index": pairs[:, 0],
            "value": pairs.view(torch.float32)[:, 1], "pairs": pairs}


def test_paired_views_are_recognised():
    d = _pair_dict()
    assert ops._paired(d)
    assert d["index"].stride(0) == 2 and d["value"].data_ptr() == d["index"].data_ptr() + 4
    # the pair views read back the values written through the pair buffer
    torch.testing.assert_close(d["value"], torch.linspace(-1, 1, 37))
    assert d["index"].tolist() == list(range(37))


def test_contiguous_or_unrelated_views_are_not_pairs():
    d = _pair_dict()
    assert not ops._paired({"offset": d["offset"], "index": d["index"].contiguous(),
                            "value": d["value"].contiguous()})
    # value from another buffer, or shifted by a whole pair
    other = torch.zeros((37, 2), dtype=torch.int32)
    assert not ops._paired({"offset": d["offset"], "index": d["index"],
                            "value": other.view(torch.float32)[:, 1]})
    assert not ops._paired({"offset": d["offset"], "index": d["pairs"][1:, 0],
                            "value": d["pairs"].view(torch.float32)[:-1, 1]})
    assert not ops._paired({"offset": d["offset"], "index": d["index"], "value": None})
    # 64-bit indices never form pairs
    p64 = torch.zeros((37, 2), dtype=torch.int64)
    assert not ops._paired({"offset": d["offset"], "index": p64[:, 0],
                            "value": p64.view(torch.float64)[:, 1]})


def test_check_rejects_cpu_and_strided_arrays():
    d = _pair_dict()
    with pytest.raises(ValueError, match="contiguous device tensor"):
        ops._check(d, pairs=True)  # CPU tensors: never a device CSR
    with pytest.raises(ValueError, match="contiguous device tensor"):
        ops._check(d)
