"""BASELINE config 5: LibFM / LibSVM -> signed feature hash -> dense fp8 batch.

* an independent numpy implementation of the K9 hash (murmur3 fmix64 of
  index ^ field << 40 mixed with the seed; bucket = h % dim, sign = bit 31)
  and an fp64 accumulation are the reference;
* the CSR path (tile parser + ops.hashed_dense, K9) and the FUSED path
  (GPUParser.parse_all_hashed: tokenize -> hash -> fp8 in one kernel, no CSR)
  must both match it: identical buckets and signs, f32 sums to 1e-6, and fp8
  equal to torch's e4m3fn cast of the reference (except at rounding ties of
  buckets that several features share, where the f32 summation order shows);
* HashedFM on the fused fp8 batch matches its fp32 reference.
"""
import numpy as np
import pytest
import torch

from dmlc_core_amd import data, ops
from dmlc_core_amd.models import HashedFM

pytestmark = pytest.mark.gpu
M64 = (1 << 64) - 1


def ref_hash(keys: np.ndarray, seed: int) -> np.ndarray:
    x = [int(k) for k in keys]
    out = np.empty(len(x), dtype=np.uint64)
    s = (seed * 0x9E3779B97F4A7C15) & M64
    for i, v in enumerate(x):
        v ^= s
        v = ((v ^ (v >> 33)) * 0xFF51AFD7ED558CCD) & M64
        v = ((v ^ (v >> 33)) * 0xC4CEB9FE1A85EC53) & M64
        v ^= v >> 33
        out[i] = v & 0xFFFFFFFF
    return out


def ref_dense(host, dim, seed, libfm):
    rows = len(host["label"])
    off = host["offset"].astype(np.int64)
    idx = host["index"].astype(np.uint64)
    val = (host["value"].astype(np.float64) if host.get("value") is not None
           else np.ones(len(idx)))
    keys = idx ^ (host["field"].astype(np.uint64) << np.uint64(40)) if libfm else idx
    h = ref_hash(keys, seed)
    bucket = (h % np.uint64(dim)).astype(np.int64)
    sign = np.where(h & np.uint64(0x80000000), -1.0, 1.0)
    rowid = np.repeat(np.arange(rows), np.diff(off))
    out = np.zeros((rows, dim), dtype=np.float64)
    np.add.at(out, (rowid, bucket), sign * val)
    share = np.zeros((rows, dim), dtype=np.int64)
    np.add.at(share, (rowid, bucket), 1)
    return out, share


@pytest.fixture(scope="module", params=["libfm", "libsvm"])
def dataset(request, tmp_path_factory):
    fmt = request.param
    p = str(tmp_path_factory.mktemp("h") / f"d.{fmt}")
    data.write_synthetic(p, 0, 1500, format=fmt, seed=9)
    host = data.GPUParser(p, format=fmt, chunk_bytes=128 * 1024).parse_all().to_host()
    return fmt, p, host


@pytest.mark.parametrize("dim,seed", [(48, 3), (64, 1), (256, 0), (1024, 7), (2048, 5)])
def test_k9_and_fused_match_independent_hash(dataset, dim, seed):
    fmt, p, host = dataset
    libfm = fmt == "libfm"
    ref, share = ref_dense(host, dim, seed, libfm)
    # CSR path: tile parser -> K9
    csr = data.csr_to_torch(data.GPUParser(p, format=fmt, chunk_bytes=128 * 1024).parse_all())
    k9 = ops.hashed_dense(csr, dim, seed=seed, fp8=False).cpu().numpy().astype(np.float64)
    # fused paths (tile kernel, and the exact per-line kernel), f32
    outs = [k9]
    for fast in (1, 0):
        fused = data.GPUParser(p, format=fmt, chunk_bytes=128 * 1024, fast_path=fast
                               ).parse_all_hashed(dim, seed=seed, fp8=False, strategy="fused")
        outs.append(fused["x"].cpu().numpy().astype(np.float64))
        np.testing.assert_array_equal(fused["label"].cpu().numpy(), host["label"])
    for got in outs:
        assert got.shape == ref.shape
        np.testing.assert_array_equal(got != 0, ref != 0)  # same buckets, no extra mass
        np.testing.assert_allclose(got, ref, rtol=1e-6, atol=1e-6)
    scale = 0.5
    f8 = data.GPUParser(p, format=fmt, chunk_bytes=128 * 1024).parse_all_hashed(
        dim, seed=seed, fp8=True, scale=scale, strategy="fused")["x"]
    assert f8.dtype == torch.float8_e4m3fn and tuple(f8.shape) == ref.shape
    want = torch.from_numpy((ref * scale).astype(np.float32)).to(torch.float8_e4m3fn)
    same = (f8.cpu().view(torch.uint8) == want.view(torch.uint8)).numpy()
    assert same[share <= 2].all()  # one or two terms: the f32 sum is exact
    assert same.mean() > 0.999


@pytest.mark.parametrize("dim", [200, 1024])
@pytest.mark.parametrize("scale", [0.3, 0.5, 1.0])
def test_fused_fp8_scales_match_k9(dataset, dim, scale):
    """the fused kernel's fp8 rows equal K9's for any scale: a power of two
    is applied per token, any other scale per column at the row flush"""
    fmt, p, host = dataset
    _, share = ref_dense(host, dim, 2, fmt == "libfm")
    csr = data.csr_to_torch(data.GPUParser(p, format=fmt, chunk_bytes=128 * 1024).parse_all())
    k9 = ops.hashed_dense(csr, dim, seed=2, fp8=True, scale=scale).cpu().view(torch.uint8)
    f8 = data.GPUParser(p, format=fmt, chunk_bytes=128 * 1024).parse_all_hashed(
        dim, seed=2, fp8=True, scale=scale, strategy="fused")["x"].cpu().view(torch.uint8)
    same = (f8 == k9).numpy()
    assert same[share <= 2].all()  # one or two terms: the f32 sums are exact
    assert same.mean() > 0.999


def test_hashed_fm_on_fused_fp8_batch(dataset):
    fmt, p, _ = dataset
    scale = 0.25
    b = data.GPUParser(p, format=fmt).parse_all_hashed(512, seed=1, fp8=True, scale=scale)
    torch.manual_seed(0)
    model = HashedFM(dim=512, rank=16).cuda()
    with torch.no_grad():
        model.w.normal_(0, 0.05)
        model.bias.fill_(0.1)
    y = model(b["x"], scale=scale)
    x = b["x"].float() / scale
    ref = HashedFM.reference(x, model.w.detach(), model.v.detach(), model.bias.detach())
    err = (y.detach() - ref).abs().max().item() / (ref.abs().max().item() + 1e-6)
    assert model.gemm == "hip_mfma_bf16"
    assert err < 0.05, (err, model.gemm)  # bf16 [w | V] operand
    loss = torch.nn.functional.binary_cross_entropy_with_logits(y, b["label"].clamp(0, 1))
    loss.backward()
    assert model.w.grad is not None and torch.isfinite(model.w.grad).all()
    assert model.v.grad is not None and torch.isfinite(model.v.grad).all()
    print("HashedFM gemm path:", model.gemm)


def test_fused_tile_kernel_long_lines(tmp_path):
    """A wave follows its tile's last line past the tile end for any length:
    lines of ~20 KB (several tiles, tiles that own no line) mixed with short
    ones stay on the tile kernel (no exact fallback) and equal K9."""
    rng = np.random.default_rng(2)
    lines = []
    for r in range(300):
        n = int(rng.integers(5, 40)) if r % 50 else 1500  # every 50th line ~ 20 KB
        toks = [f"{int(rng.integers(0, 30))}:{int(rng.integers(0, 1 << 20))}:{rng.random():.4f}"
                for _ in range(n)]
        lines.append(f"{r % 2} " + " ".join(toks))
    p = str(tmp_path / "long.libfm")
    with open(p, "w") as f:
        f.write("\n".join(lines) + "\n")
    g = data.GPUParser(p, format="libfm", chunk_bytes=256 * 1024)
    fused = g.parse_all_hashed(256, seed=3, fp8=False)
    assert g.stats()["exact_chunks"] == 0
    csr = data.csr_to_torch(data.GPUParser(p, format="libfm").parse_all())
    k9 = ops.hashed_dense(csr, 256, seed=3, fp8=False)
    np.testing.assert_allclose(fused["x"].cpu().numpy(), k9.cpu().numpy(), rtol=1e-5, atol=1e-5)
    np.testing.assert_array_equal(fused["label"].cpu().numpy(), csr["label"].cpu().numpy())


@pytest.mark.parametrize("fmt", ["libsvm", "libfm"])
@pytest.mark.parametrize("eol", ["\n", "\r\n"])
def test_fused_tile_kernel_line_shapes(tmp_path, fmt, eol):
    """label-only rows, runs of tiny lines (many rows per decode round), blank
    lines, exponent / long-mantissa values (generic token path), CRLF, and a
    last line without EOL: fused == exact per-line kernel == K9."""
    rng = np.random.default_rng(7)
    lines = []
    for r in range(4000):
        k = r % 7
        lab = f"{r % 3 - 1}"
        if k == 0:
            lines.append(lab)  # label only
        elif k == 1:
            lines.append("")  # blank line (no row)
            continue
        n = 1 if k == 2 else int(rng.integers(1, 30))
        toks = []
        for _ in range(n):
            i = int(rng.integers(0, 1 << 22))
            v = [f"{rng.random():.6f}", f"{rng.random():.3e}", f"{rng.random():.12f}", "7"][r % 4]
            toks.append(f"{i}:{v}" if fmt == "libsvm" else f"{int(rng.integers(0, 9))}:{i}:{v}")
        lines.append(lab + " " + " ".join(toks))
    p = str(tmp_path / f"s.{fmt}")
    with open(p, "w", newline="") as f:
        f.write(eol.join(lines))  # no EOL after the last line
    fused = data.GPUParser(p, format=fmt, chunk_bytes=64 * 1024).parse_all_hashed(
        192, seed=5, fp8=False, strategy="fused")
    exact = data.GPUParser(p, format=fmt, chunk_bytes=64 * 1024, fast_path=0).parse_all_hashed(
        192, seed=5, fp8=False, strategy="fused")
    csr = data.csr_to_torch(data.GPUParser(p, format=fmt, chunk_bytes=64 * 1024).parse_all())
    k9 = ops.hashed_dense(csr, 192, seed=5, fp8=False).cpu().numpy()
    np.testing.assert_array_equal(fused["label"].cpu().numpy(), exact["label"].cpu().numpy())
    np.testing.assert_array_equal(fused["label"].cpu().numpy(), csr["label"].cpu().numpy())
    np.testing.assert_allclose(fused["x"].cpu().numpy(), exact["x"].cpu().numpy(), rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(fused["x"].cpu().numpy(), k9, rtol=1e-6, atol=1e-6)


def test_fused_batch_reuse(dataset):
    """out=<earlier result> refills the same HBM buffers (no new allocation)
    and yields the same batch; a different dim reallocates."""
    fmt, p, _ = dataset
    g = data.GPUParser(p, format=fmt, chunk_bytes=128 * 1024, hbm_cache=1)
    a = g.parse_all_hashed(1024, seed=4)
    want = a["x"].view(torch.uint8).clone()
    ptr = a["x"].data_ptr()
    for _ in range(2):
        g.before_first()
        b = g.parse_all_hashed(1024, seed=4, out=a)
        assert b is a  # same shape: the tensors already alias the refilled batch
        assert b["x"].data_ptr() == ptr
        assert torch.equal(b["x"].view(torch.uint8), want)
    g.before_first()
    c = g.parse_all_hashed(256, seed=4, out=b)
    assert tuple(c["x"].shape) == (want.shape[0], 256)
    # the reshape reallocated: the earlier tensors keep their own buffers
    # (each DLPack capsule owns what it exports), still readable, unchanged
    torch.cuda.synchronize()
    assert b["x"].data_ptr() == ptr
    assert torch.equal(b["x"].view(torch.uint8), want)


@pytest.mark.parametrize("fmt,junk", [("libsvm", "0 junk 3:1\n1 qid:4 5:1\n"),
                                      ("libfm", "1 x:2:1 1:3:0.5\n0 #c 2:2:1\n")])
def test_fused_tile_kernel_bad_token_starts_fall_back(tmp_path, fmt, junk):
    """Token starts outside [0-9+-.] are flagged by the fused kernel itself
    (the count pass no longer checks them): the chunk takes the exact per-line
    kernel and the batch equals the all-exact run."""
    p = str(tmp_path / f"j.{fmt}")
    data.write_synthetic(p, 0, 600, format=fmt, seed=4)
    with open(p, "a") as f:
        f.write(junk)
    data.write_synthetic(str(tmp_path / "t"), 600, 1200, format=fmt, seed=4)
    with open(p, "a") as f:
        f.write(open(str(tmp_path / "t")).read())
    g = data.GPUParser(p, format=fmt, chunk_bytes=32 * 1024)
    fused = g.parse_all_hashed(256, seed=2, fp8=False, strategy="fused")
    assert 0 < g.stats()["exact_chunks"] < g.stats()["chunks"]
    exact = data.GPUParser(p, format=fmt, chunk_bytes=32 * 1024, fast_path=0).parse_all_hashed(
        256, seed=2, fp8=False, strategy="fused")
    np.testing.assert_array_equal(fused["label"].cpu().numpy(), exact["label"].cpu().numpy())
    np.testing.assert_allclose(fused["x"].cpu().numpy(), exact["x"].cpu().numpy(), rtol=1e-6,
                               atol=1e-6)


@pytest.mark.parametrize("dim", [256, 1024])
def test_hashed_strategies_agree(dataset, dim):
    """auto / csr / fused return the same batch (f32: exact up to the order of
    colliding terms) and the same labels."""
    fmt, p, host = dataset
    got = {}
    for strat in ("auto", "csr", "fused"):
        got[strat] = data.GPUParser(p, format=fmt, chunk_bytes=128 * 1024).parse_all_hashed(
            dim, seed=2, fp8=False, strategy=strat)
        np.testing.assert_array_equal(got[strat]["label"].cpu().numpy(), host["label"])
    for strat in ("auto", "fused"):
        np.testing.assert_allclose(got[strat]["x"].cpu().numpy(), got["csr"]["x"].cpu().numpy(),
                                   rtol=1e-6, atol=1e-6)
    with pytest.raises(ValueError):
        data.GPUParser(p, format=fmt).parse_all_hashed(dim, strategy="nope")


@pytest.mark.parametrize("dim,rows", [(128, 37), (512, 1000), (1024, 4133)])
def test_fm_kernels_match_fp32(dim, rows):
    """F1 / F2 (bf16 MFMA over the fp8 batch) against fp32 autograd of the same
    model: x is exact in bf16, [w | V] is rounded to bf16 for the x.[w | V]
    product (the kernel's operand), x^2.q and the epilogue stay f32; the
    backward's G = [g, g xV] operand is bf16, hence the looser gradient bound."""
    torch.manual_seed(dim + rows)
    dev = "cuda"
    x8 = (torch.randn(rows, dim, device=dev) * 2).to(torch.float8_e4m3fn)
    x8[:, ::7] = 0  # sparse-ish, like a hashed batch
    scale = 0.5
    model = HashedFM(dim=dim, rank=16).to(dev)
    with torch.no_grad():
        model.w.normal_(0, 0.05)
        model.v.normal_(0, 0.05)
        model.bias.fill_(0.3)
    r = torch.randn(rows, device=dev)
    y = model(x8, scale=scale)
    assert model.gemm == "hip_mfma_bf16"
    (y * r).sum().backward()
    x = x8.float() / scale
    w = model.w.detach().clone().requires_grad_(True)
    v = model.v.detach().clone().requires_grad_(True)
    b = model.bias.detach().clone().requires_grad_(True)
    wb = w.detach().to(torch.bfloat16).float() + (w - w.detach())  # bf16 values, fp32 grads
    vb = v.detach().to(torch.bfloat16).float() + (v - v.detach())
    xv = x @ vb
    ref = b + (x @ wb).squeeze(-1) + 0.5 * ((xv ** 2).sum(-1) - (x ** 2) @ (v ** 2).sum(1))
    (ref * r).sum().backward()
    tol = ref.detach().abs().max().item()
    assert (y.detach() - ref.detach()).abs().max().item() <= 1e-4 * tol + 1e-5
    for got, want in ((model.w.grad, w.grad), (model.v.grad, v.grad), (model.bias.grad, b.grad)):
        err = (got - want).abs().max().item() / (want.abs().max().item() + 1e-6)
        assert err < 2e-2, err


@pytest.mark.parametrize("dim,rows,kind,weighted", [
    (128, 37, "logistic", False), (256, 1000, "squared", True), (512, 3001, "logistic", True),
    (1024, 4133, "logistic", False), (1024, 70000, "squared", False)])
def test_fm_fused_step_matches_two_pass(dim, rows, kind, weighted):
    """F5 (forward + loss + backward in one pass over the batch) against the
    two-pass path (F1, torch loss, F2) and the fp32 reference: the same loss
    and logits (f32 epilogues), gradients within the bf16-G bound of
    test_fm_kernels_match_fp32."""
    torch.manual_seed(dim + rows)
    dev = "cuda"
    x8 = (torch.randn(rows, dim, device=dev) * 2).to(torch.float8_e4m3fn)
    x8[:, ::5] = 0
    scale = 0.5
    label = (torch.rand(rows, device=dev) > 0.5).float()
    weight = torch.rand(rows, device=dev) + 0.5 if weighted else None
    model = HashedFM(dim=dim, rank=16).to(dev)
    with torch.no_grad():
        model.w.normal_(0, 0.05)
        model.v.normal_(0, 0.05)
        model.bias.fill_(0.1)
    fused = model.loss(x8, label, scale=scale, loss=kind, weight=weight)
    assert model.gemm == "hip_mfma_bf16_fused"
    fused.backward()
    got = [p.grad.clone() for p in (model.w, model.v, model.bias)]
    logits = model.last_logits.clone()
    model.zero_grad()
    y = model(x8, scale=scale)
    if kind == "logistic":
        ref = torch.nn.functional.binary_cross_entropy_with_logits(y, label, weight=weight)
    else:
        e = (y - label) ** 2
        ref = (e * weight).mean() if weighted else e.mean()
    ref.backward()
    want = [p.grad.clone() for p in (model.w, model.v, model.bias)]
    # the same f32 epilogue over partial sums added in another order (the
    # fused step splits K over the workgroup's waves): the F1 test's bound
    tol = y.detach().abs().max().item()
    assert (logits - y.detach()).abs().max().item() <= 1e-4 * tol + 1e-5
    assert abs(fused.item() - ref.item()) <= 1e-4 * abs(ref.item()) + 1e-6
    for g, w in zip(got, want):
        err = (g - w).abs().max().item() / (w.abs().max().item() + 1e-9)
        assert err < 1e-2, err
    # and against fp32 autograd of the same model
    x = x8.float() / scale
    w32 = model.w.detach().clone().requires_grad_(True)
    v32 = model.v.detach().clone().requires_grad_(True)
    b32 = model.bias.detach().clone().requires_grad_(True)
    y32 = HashedFM.reference(x, w32, v32, b32)
    if kind == "logistic":
        l32 = torch.nn.functional.binary_cross_entropy_with_logits(y32, label, weight=weight)
    else:
        e = (y32 - label) ** 2
        l32 = (e * weight).mean() if weighted else e.mean()
    l32.backward()
    for g, w in zip(got, (w32.grad, v32.grad, b32.grad)):
        err = (g - w).abs().max().item() / (w.abs().max().item() + 1e-9)
        assert err < 2e-2, err


@pytest.mark.parametrize("extra", [1, 33])
def test_fm_fused_empty_trailing_blocks(extra):
    """rows just above 32 x CUs: the per-block row count rounds up to 64, so
    the last workgroups start at or past the last row.  They must load only
    inside the batch (the clamp row is rows - 1, not their own start) and
    add nothing: the loss and gradients equal the two-pass path's."""
    torch.manual_seed(extra)
    dev = "cuda"
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    rows, dim = 32 * cus + extra, 256
    # the batch sits at the end of its own allocation (no slack after it)
    x8 = (torch.randn(rows, dim, device=dev) * 2).to(torch.float8_e4m3fn).clone()
    label = (torch.rand(rows, device=dev) > 0.5).float()
    model = HashedFM(dim=dim, rank=16).to(dev)
    with torch.no_grad():
        model.w.normal_(0, 0.05)
        model.v.normal_(0, 0.05)
    fused = model.loss(x8, label, loss="squared")
    assert model.gemm == "hip_mfma_bf16_fused"
    fused.backward()
    got = [p.grad.clone() for p in (model.w, model.v, model.bias)]
    model.zero_grad()
    y = model(x8)
    ref = ((y - label) ** 2).mean()
    ref.backward()
    assert abs(fused.item() - ref.item()) <= 1e-4 * abs(ref.item()) + 1e-6
    for g, p in zip(got, (model.w, model.v, model.bias)):
        err = (g - p.grad).abs().max().item() / (p.grad.abs().max().item() + 1e-9)
        assert err < 1e-2, err


def test_fm_fused_step_trains():
    """A few SGD steps of the fused path lower the loss (the gradient signs
    and the mean scaling are right end to end)."""
    torch.manual_seed(0)
    dev = "cuda"
    rows, dim = 8192, 256
    x8 = (torch.randn(rows, dim, device=dev)).to(torch.float8_e4m3fn)
    truth = torch.randn(dim, device=dev) * 0.3
    label = ((x8.float() @ truth) > 0).float()
    model = HashedFM(dim=dim, rank=16).to(dev)
    opt = torch.optim.SGD(model.parameters(), lr=0.5)
    losses = []
    for _ in range(20):
        opt.zero_grad()
        loss = model.loss(x8, label)
        loss.backward()
        opt.step()
        losses.append(loss.item())
    assert losses[-1] < 0.8 * losses[0], losses


@pytest.mark.parametrize("fmt", ["libsvm", "libfm"])
def test_one_pass_hashed_matches_counted(tmp_path, fmt):
    """With ``hash_one_pass=1`` a replayed pass into a reused batch runs one
    kernel per chunk (line counts by decoupled look-back, no count kernel;
    the default is the counted kernel, measured faster): the same fp8 bytes and
    labels as the counted first pass; a batch too small for the partition
    overflows, grows and the chunk is written again."""
    p = str(tmp_path / f"big.{fmt}")
    data.write_synthetic(p, 0, 30000, format=fmt, seed=11)
    g = data.GPUParser(p, format=fmt, chunk_bytes=1 << 20, hbm_cache=1, hash_one_pass=1)
    a = g.parse_all_hashed(512, seed=6)  # first pass: caching, C1 + C2 + hash
    want_x = a["x"].view(torch.uint8).clone()
    want_l = a["label"].clone()
    assert g.stats()["one_pass_chunks"] == 0
    g.before_first()
    b = g.parse_all_hashed(512, seed=6, out=a)  # resident: one pass, merged chunks
    assert g.stats()["one_pass_chunks"] >= 1
    assert torch.equal(b["x"].view(torch.uint8), want_x)
    assert torch.equal(b["label"], want_l)
    small_p = str(tmp_path / f"small.{fmt}")
    data.write_synthetic(small_p, 0, 50, format=fmt, seed=2)
    small = data.GPUParser(small_p, format=fmt).parse_all_hashed(512, seed=6)
    assert small["x"].shape[0] == 50
    g.before_first()
    c = g.parse_all_hashed(512, seed=6, out=small)
    assert tuple(c["x"].shape) == tuple(want_x.shape)
    assert torch.equal(c["x"].view(torch.uint8), want_x)
    assert torch.equal(c["label"], want_l)


@pytest.mark.parametrize("bad", ["0 1:1\n 1 2:1\n", "1 3:1\x0b 4:1\n"])
def test_one_pass_hashed_irregular_falls_back(tmp_path, bad):
    """Blank-started lines and stray control bytes, which the count kernel
    flags on the counted pass, are flagged by the one-pass kernel itself: the
    chunk takes the exact kernels and the batch equals the counted pass."""
    p = str(tmp_path / "irr.libsvm")
    data.write_synthetic(p, 0, 8000, format="libsvm", seed=5)
    with open(p, "a") as f:
        f.write(bad)
    data.write_synthetic(str(tmp_path / "t"), 8000, 16000, format="libsvm", seed=5)
    with open(p, "a") as f:
        f.write(open(str(tmp_path / "t")).read())
    g = data.GPUParser(p, format="libsvm", chunk_bytes=1 << 20, hbm_cache=1, hash_one_pass=1)
    a = g.parse_all_hashed(256, seed=3, fp8=False)
    want_x, want_l = a["x"].clone(), a["label"].clone()
    e0 = g.stats()["exact_chunks"]
    assert e0 >= 1
    g.before_first()
    b = g.parse_all_hashed(256, seed=3, fp8=False, out=a)
    assert g.stats()["exact_chunks"] > e0
    np.testing.assert_array_equal(b["label"].cpu().numpy(), want_l.cpu().numpy())
    np.testing.assert_allclose(b["x"].cpu().numpy(), want_x.cpu().numpy(), rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("width", [2, 1])
def test_fused_hash_dense_token_steps(tmp_path, width):
    """Steps with more tokens than the hash kernel's list (valueless 2-digit
    LibSVM features: ~680 tokens per 2 KiB step) are listed and decoded in
    two halves; 1-digit ones (~1000 per step) go to the exact kernels.  Both
    equal the all-exact batch."""
    rng = np.random.default_rng(width)
    lo, hi = (10, 100) if width == 2 else (1, 10)
    lines = []
    for i in range(3000):
        feats = " ".join(str(v) for v in rng.integers(lo, hi, size=int(rng.integers(1, 60))))
        lines.append(f"{i % 2} {feats}\n")
    p = str(tmp_path / "dense.libsvm")
    with open(p, "w") as f:
        f.writelines(lines)
    g = data.GPUParser(p, format="libsvm", chunk_bytes=64 * 1024)
    fused = g.parse_all_hashed(256, seed=8, fp8=False, strategy="fused")
    if width == 2:
        assert g.stats()["exact_chunks"] == 0
    exact = data.GPUParser(p, format="libsvm", chunk_bytes=64 * 1024, fast_path=0).parse_all_hashed(
        256, seed=8, fp8=False, strategy="fused")
    np.testing.assert_array_equal(fused["label"].cpu().numpy(), exact["label"].cpu().numpy())
    np.testing.assert_allclose(fused["x"].cpu().numpy(), exact["x"].cpu().numpy(), rtol=1e-6,
                               atol=1e-6)
