"""HIP feature kernels (K9 hashed dense f32/fp8, K11 SpMV / SpMV^T) against
plain PyTorch fp32 references of the same ops, and one autograd step of the
sparse logistic-regression model."""
import numpy as np
import pytest

from dmlc_core_amd import data, ops

pytestmark = pytest.mark.gpu


@pytest.fixture
def csr_t(tmp_path):
    p = str(tmp_path / "s.libsvm")
    data.write_synthetic(p, 0, 3000, seed=1, num_features=5000)
    csr = data.GPUParser(p).parse_all()
    return data.csr_to_torch(csr), csr


def dense_ref(t, nfeat):
    import torch
    off = t["offset"].cpu().numpy().astype(np.int64)
    idx = t["index"].cpu().numpy().astype(np.int64)
    val = t["value"].cpu().numpy()
    rows = np.repeat(np.arange(len(off) - 1), np.diff(off))
    x = torch.zeros((len(off) - 1, nfeat), dtype=torch.float32)
    x.index_put_((torch.from_numpy(rows), torch.from_numpy(idx)), torch.from_numpy(val), accumulate=True)
    return x


def test_spmv_matches_torch(csr_t):
    import torch
    t, csr = csr_t
    nfeat = int(csr.max_index) + 1
    w = torch.randn(nfeat, device="cuda")
    y = ops.spmv(t, w, 0.5)
    x = dense_ref(t, nfeat)
    ref = x @ w.cpu() + 0.5
    torch.testing.assert_close(y.cpu(), ref, rtol=1e-5, atol=1e-4)


def test_spmv_t_matches_torch(csr_t):
    import torch
    t, csr = csr_t
    nfeat = int(csr.max_index) + 1
    d = torch.randn(csr.rows, device="cuda")
    g = ops.spmv_t(t, d, nfeat)
    x = dense_ref(t, nfeat)
    torch.testing.assert_close(g.cpu(), x.t() @ d.cpu(), rtol=1e-4, atol=1e-4)


def test_hashed_dense_f32_and_fp8(csr_t):
    import torch
    t, csr = csr_t
    f32 = ops.hashed_dense(t, 512, seed=3, fp8=False)
    assert f32.shape == (csr.rows, 512)
    # every row's hashed mass equals its signed value sum in magnitude bound
    vals = t["value"].cpu().numpy()
    off = t["offset"].cpu().numpy().astype(np.int64)
    l1 = np.add.reduceat(np.abs(vals), off[:-1])
    assert np.all(np.abs(f32.cpu().numpy()).sum(1) <= l1 + 1e-4)
    fp8 = ops.hashed_dense(t, 512, seed=3, fp8=True)
    assert fp8.dtype == torch.float8_e4m3fn
    ref = f32.cpu().to(torch.float8_e4m3fn).float()
    torch.testing.assert_close(fp8.cpu().float(), ref, rtol=0, atol=0)


def test_logreg_step_decreases_loss(csr_t):
    import torch
    from dmlc_core_amd.models import SparseLogReg
    t, csr = csr_t
    model = SparseLogReg(int(csr.max_index) + 1).cuda()
    opt = torch.optim.SGD(model.parameters(), lr=0.5)
    losses = []
    for _ in range(5):
        opt.zero_grad()
        loss = model.loss(t)
        loss.backward()
        opt.step()
        losses.append(float(loss))
    assert losses[-1] < losses[0]


def test_transpose_and_gather_gradient_match(csr_t):
    """ops.transpose (device sort -> CSC) and the gather gradient agree with
    the dense reference and with the atomic SpMV^T; autograd through both
    gradient modes gives the same weights' gradient."""
    import torch
    from dmlc_core_amd.models import SparseLogReg
    t, csr = csr_t
    nfeat = int(csr.max_index) + 1 + 7  # trailing features nobody uses
    tt = ops.transpose(t, nfeat)
    assert tt["offset"].numel() == nfeat + 1 and int(tt["offset"][-1]) == t["index"].numel()
    d = torch.randn(csr.rows, device="cuda")
    x = dense_ref(t, nfeat)
    g = ops.spmv(tt, d, 0.0)
    torch.testing.assert_close(g.cpu(), x.t() @ d.cpu(), rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(g, ops.spmv_t(t, d, nfeat), rtol=1e-4, atol=1e-4)
    grads = {}
    for mode in ("transpose", "atomic"):
        m = SparseLogReg(nfeat, grad=mode).cuda()
        with torch.no_grad():
            m.weight.normal_(0, 0.1)
            m.weight.copy_(torch.linspace(-1, 1, nfeat, device="cuda"))
        m.loss(t).backward()
        grads[mode] = m.weight.grad.clone()
    assert "transpose" in t  # cached for the next step
    torch.testing.assert_close(grads["transpose"], grads["atomic"], rtol=1e-4, atol=1e-6)


def test_transposed_dict_feeds_every_op(csr_t):
    """A transpose's (paired) dict is a CSR like any other: spmv_t,
    hashed_dense and transpose take it (unpaired into contiguous copies), and
    transposing twice gives back the original CSR."""
    import torch
    t, csr = csr_t
    nfeat = int(csr.max_index) + 1
    tt = ops.transpose(t, nfeat)
    assert ops._paired(tt)
    xt = dense_ref({k: tt[k] for k in ("offset", "index", "value")}, csr.rows)
    w = torch.randn(nfeat, device="cuda")
    torch.testing.assert_close(ops.spmv_t(tt, w, csr.rows).cpu(), xt.t() @ w.cpu(),
                               rtol=1e-4, atol=1e-4)
    contig = {"offset": tt["offset"], "index": tt["index"].contiguous(),
              "value": tt["value"].contiguous()}
    torch.testing.assert_close(ops.hashed_dense(tt, 256, seed=1, fp8=False),
                               ops.hashed_dense(contig, 256, seed=1, fp8=False), rtol=0, atol=0)
    back = ops.transpose(tt, csr.rows)
    np.testing.assert_array_equal(back["offset"].cpu().numpy(),
                                  t["offset"].cpu().numpy().astype(np.int64))
    torch.testing.assert_close(dense_ref(back, nfeat), dense_ref(t, nfeat), rtol=0, atol=0)


def test_transpose_workspace_is_persistent_and_out_reuses(csr_t):
    """The sort's scratch is kept between builds (no multi-GB allocation per
    build); out= overwrites a previous result; both give the same CSC as a
    fresh build, and release_workspace() frees the scratch."""
    import torch
    t, csr = csr_t
    nfeat = int(csr.max_index) + 1
    a = ops.transpose(t, nfeat)
    ws = [w.data_ptr() for w in ops._WORKSPACE.values()]
    assert ws
    b = ops.transpose(t, nfeat)
    assert [w.data_ptr() for w in ops._WORKSPACE.values()] == ws
    for k in ("offset", "index", "value"):
        torch.testing.assert_close(a[k], b[k], rtol=0, atol=0)
    junk = {k: torch.full_like(v, 7) for k, v in a.items()}
    c = ops.transpose(t, nfeat, out=junk)
    assert c["index"].data_ptr() == junk["index"].data_ptr()
    for k in ("offset", "index", "value"):
        torch.testing.assert_close(a[k], c[k], rtol=0, atol=0)
    with pytest.raises(ValueError, match="out= does not fit"):
        ops.transpose(t, nfeat + 1, out=junk)
    # a previous (paired) result as out=: the pairs are overwritten in place
    a["pairs"].fill_(7)
    d = ops.transpose(t, nfeat, out=a)
    assert d["pairs"].data_ptr() == a["pairs"].data_ptr()
    for k in ("offset", "index", "value"):
        torch.testing.assert_close(b[k], d[k], rtol=0, atol=0)
    ops.release_workspace()
    assert not ops._WORKSPACE


def test_transpose_of_a_row_slice_and_auto_mode(csr_t):
    """A batch that is a row slice of a larger CSR (offsets not starting at 0,
    full index / value arrays -- examples/train_sparse_logreg.py) transposes to
    the slice's own entries; grad="auto" uses atomics on a dict's first
    backward and the cached transpose from the second on."""
    import torch
    from dmlc_core_amd.models import SparseLogReg
    t, csr = csr_t
    nfeat = int(csr.max_index) + 1
    x = dense_ref(t, nfeat)
    b, e = 1000, 1700
    batch = {"offset": t["offset"][b:e + 1], "index": t["index"], "value": t["value"]}
    d = torch.randn(e - b, device="cuda")
    g = ops.spmv(ops.transpose(batch, nfeat), d, 0.0)
    torch.testing.assert_close(g.cpu(), x[b:e].t() @ d.cpu(), rtol=1e-4, atol=1e-4)
    m = SparseLogReg(nfeat).cuda()  # grad="auto"
    holder = {"offset": t["offset"][b:e + 1], "index": t["index"], "value": t["value"],
              "label": t["label"][b:e]}
    grads = []
    for _ in range(3):
        m.zero_grad()
        m.loss(holder).backward()
        grads.append(m.weight.grad.clone())
        if _ == 0:
            assert "transpose" not in holder
    assert "transpose" in holder
    torch.testing.assert_close(grads[1], grads[0], rtol=1e-4, atol=1e-6)


def test_cached_transpose_follows_the_dict_tensors(csr_t):
    """A dict refilled with another batch's tensors (csr.update(next_batch))
    must not reuse the transpose of the previous tensors: every backward
    equals the atomic gradient of the tensors the dict holds now."""
    import torch
    from dmlc_core_amd.models import SparseLogReg
    t, csr = csr_t
    nfeat = int(csr.max_index) + 1
    m = SparseLogReg(nfeat, grad="transpose").cuda()
    ref = SparseLogReg(nfeat, grad="atomic").cuda()
    with torch.no_grad():
        m.weight.copy_(torch.linspace(-1, 1, nfeat, device="cuda"))
        ref.weight.copy_(m.weight)
    holder = {}
    for b, e in ((0, 900), (900, 2000), (300, 1300)):
        batch = {"offset": t["offset"][b:e + 1].clone(), "index": t["index"], "value": t["value"],
                 "label": t["label"][b:e].clone()}
        holder.update(batch)
        m.zero_grad()
        ref.zero_grad()
        m.loss(holder).backward()
        ref.loss(batch).backward()
        torch.testing.assert_close(m.weight.grad, ref.weight.grad, rtol=1e-4, atol=1e-6)
    # an in-place rewrite of the values invalidates it too
    holder["value"] = t["value"].clone()
    m.zero_grad()
    m.loss(holder).backward()
    holder["value"].mul_(2.0)
    m.zero_grad()
    ref.zero_grad()
    m.loss(holder).backward()
    ref.loss({k: holder[k] for k in ("offset", "index", "value", "label")}).backward()
    torch.testing.assert_close(m.weight.grad, ref.weight.grad, rtol=1e-4, atol=1e-6)


def _ref_transpose(t, nfeat):
    off = t["offset"].cpu().numpy().astype(np.int64)
    lo, hi = off[0], off[-1]
    idx = t["index"].cpu().numpy().astype(np.int64)[lo:hi]
    val = t["value"].cpu().numpy()[lo:hi]
    rows = np.repeat(np.arange(len(off) - 1), np.diff(off))
    order = np.argsort(idx, kind="stable")  # stable: rows ascending within a column
    ptr = np.searchsorted(idx[order], np.arange(nfeat + 1))
    return ptr, rows[order].astype(np.int32), val[order]


@pytest.mark.parametrize("nfeat,rows,index64", [(5000, 3000, False), (1 << 22, 20000, False),
                                                  (70000, 5000, True), (1, 50, False),
                                                  ((1 << 22) + 1, 20000, False),
                                                  (1 << 24, 20000, False), (1 << 26, 20000, False),
                                                  (1 << 26, 5000, True)])
def test_transpose_kernel_is_a_stable_csc(tmp_path, nfeat, rows, index64):
    """the HIP counting-sort transpose equals numpy's stable argsort CSC
    exactly (row ids ascending within every column, values moved with them),
    across bucket counts (1 .. 1024 buckets of 1024 - 4096 columns), the
    three-level sort of wider feature spaces (2^22 + 1 .. 2^26 columns:
    buckets of 2^16 .. 2^18 columns, 256-column super-buckets), 64-bit
    indices, and a single column"""
    p = str(tmp_path / "t.libsvm")
    data.write_synthetic(p, 0, rows, seed=5, num_features=nfeat, min_nnz=1, max_nnz=40)
    t = data.csr_to_torch(data.GPUParser(p, index64=index64).parse_all(data.DeviceCSR(index64)))
    tt = ops.transpose(t, nfeat)
    ptr, r, v = _ref_transpose(t, nfeat)
    np.testing.assert_array_equal(tt["offset"].cpu().numpy(), ptr)
    np.testing.assert_array_equal(tt["index"].cpu().numpy(), r)
    np.testing.assert_array_equal(tt["value"].cpu().numpy(), v)
    # values: index / value are the columns of one interleaved pair buffer
    assert tt["index"].stride(0) == 2 and tt["value"].stride(0) == 2
    assert tt["value"].data_ptr() == tt["index"].data_ptr() + 4
    assert tt["pairs"].shape[1] == 2


def test_spmv_over_pairs_matches_separate_arrays(csr_t):
    """K11 over a transpose's interleaved (index, value) pairs equals K11 over
    contiguous copies of the same arrays and the fp32 dense reference; the
    other ops take the strided views too (unpaired into copies)"""
    import torch
    t, csr = csr_t
    nfeat = int(csr.max_index) + 1
    tt = ops.transpose(t, nfeat)
    assert ops._paired(tt)
    sep = {"offset": tt["offset"], "index": tt["index"].contiguous(),
           "value": tt["value"].contiguous()}
    assert not ops._paired(sep)
    d = torch.randn(csr.rows, device="cuda")
    g_pairs = ops.spmv(tt, d, 0.5)
    g_sep = ops.spmv(sep, d, 0.5)
    torch.testing.assert_close(g_pairs, g_sep, rtol=0, atol=0)
    x = dense_ref(t, nfeat)
    torch.testing.assert_close(g_pairs.cpu(), x.t() @ d.cpu() + 0.5, rtol=1e-4, atol=1e-4)
    w = torch.randn(nfeat, device="cuda")
    # (f32 atomics: the summation order varies)
    torch.testing.assert_close(ops.spmv_t(tt, w, csr.rows), ops.spmv_t(sep, w, csr.rows),
                               rtol=1e-5, atol=1e-5)


def test_transpose_with_long_runs_of_empty_rows():
    """rows found for entries after > 64 empty rows (the T3 row window moves
    on past them) and after rows that end exactly at group boundaries: the
    CSC equals numpy's stable argsort"""
    import torch
    rng = np.random.default_rng(11)
    lens = rng.integers(1, 9, size=5000)
    lens[100:400] = 0          # 300 empty rows in a row
    lens[1000:1065] = 0        # exactly 65
    lens[2000:2064] = 0        # exactly 64
    lens[3000] = 64            # a row of exactly one 64-entry group
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    nfeat = 3000
    idx = rng.integers(0, nfeat, size=int(off[-1])).astype(np.int32)
    val = rng.standard_normal(int(off[-1])).astype(np.float32)
    t = {"offset": torch.from_numpy(off).cuda(), "index": torch.from_numpy(idx).cuda(),
         "value": torch.from_numpy(val).cuda()}
    tt = ops.transpose(t, nfeat)
    ptr, r, v = _ref_transpose(t, nfeat)
    np.testing.assert_array_equal(tt["offset"].cpu().numpy(), ptr)
    np.testing.assert_array_equal(tt["index"].cpu().numpy(), r)
    np.testing.assert_array_equal(tt["value"].cpu().numpy(), v)


def test_transpose_rejects_out_of_range_ids(csr_t):
    t, csr = csr_t
    with pytest.raises(ValueError, match="num_features"):
        ops.transpose(t, int(csr.max_index))  # the largest id is out of range
    from dmlc_core_amd import _dmlc
    assert _dmlc.csr_transpose_max_features() == 1 << 28
    with pytest.raises(ValueError):
        ops.transpose(t, _dmlc.csr_transpose_max_features() + 1)


def test_wide_model_auto_grad_uses_the_three_level_transpose(tmp_path):
    """SparseLogReg(2^24) under grad='auto' builds the (three-level) transpose
    on the first backward of a whole CSR; the gradient equals the atomic
    form.  A CSR without values transposes to the same rows."""
    import torch
    from dmlc_core_amd.models import SparseLogReg
    nfeat = 1 << 24
    p = str(tmp_path / "w.libsvm")
    data.write_synthetic(p, 0, 8000, seed=9, num_features=nfeat, min_nnz=1, max_nnz=30)
    t = data.csr_to_torch(data.GPUParser(p).parse_all())
    m = SparseLogReg(nfeat).cuda()
    with torch.no_grad():
        m.weight.normal_(0, 0.1)
    m.loss(t).backward()
    assert "transpose" in t
    a = SparseLogReg(nfeat, grad="atomic").cuda()
    with torch.no_grad():
        a.weight.copy_(m.weight)
        a.bias.copy_(m.bias)
    a.loss({k: v for k, v in t.items() if k in ("offset", "index", "value", "label")}).backward()
    torch.testing.assert_close(m.weight.grad, a.weight.grad, rtol=1e-4, atol=1e-6)
    novals = {"offset": t["offset"], "index": t["index"]}
    tt = ops.transpose(novals, nfeat)
    assert tt["value"] is None
    ptr, r, _ = _ref_transpose(t, nfeat)
    np.testing.assert_array_equal(tt["offset"].cpu().numpy(), ptr)
    np.testing.assert_array_equal(tt["index"].cpu().numpy(), r)


def test_auto_grad_builds_the_transpose_on_a_whole_csr(csr_t):
    """grad='auto': a whole CSR (csr_to_torch) gets its transpose on the
    first backward; the gradient equals the atomic form"""
    import torch
    from dmlc_core_amd.models import SparseLogReg
    t, csr = csr_t
    nfeat = int(csr.max_index) + 1
    m = SparseLogReg(nfeat).cuda()
    m.loss(t).backward()
    assert "transpose" in t
    a = SparseLogReg(nfeat, grad="atomic").cuda()
    with torch.no_grad():
        a.weight.copy_(m.weight)
        a.bias.copy_(m.bias)
    a.loss({k: v for k, v in t.items() if k in ("offset", "index", "value", "label")}).backward()
    torch.testing.assert_close(m.weight.grad, a.weight.grad, rtol=1e-4, atol=1e-6)


def test_auto_grad_above_the_transpose_limit_stays_atomic(csr_t):
    """grad='auto' on a model wider than the counting-sort transpose takes
    (2^28 + 1 columns): backward keeps the atomic scatter instead of raising,
    twice (the second-backward rule must not build it either), and the
    gradient equals grad='atomic'"""
    import torch
    from dmlc_core_amd import _dmlc
    from dmlc_core_amd.models import SparseLogReg
    t, _ = csr_t
    wide = _dmlc.csr_transpose_max_features() + 1
    m = SparseLogReg(wide).cuda()
    for _ in range(2):
        m.zero_grad()
        m.loss(t).backward()
    assert "transpose" not in t
    a = SparseLogReg(wide, grad="atomic").cuda()
    with torch.no_grad():
        a.weight.copy_(m.weight)
        a.bias.copy_(m.bias)
    a.loss({k: v for k, v in t.items() if k in ("offset", "index", "value", "label")}).backward()
    torch.testing.assert_close(m.weight.grad, a.weight.grad, rtol=1e-4, atol=1e-6)
