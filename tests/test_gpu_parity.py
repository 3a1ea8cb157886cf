"""GPU parity: the HIP path (through the C-ABI) against the CPU oracle.

Bit-exact comparisons on seeded inputs at sizes the oracle finishes in
seconds, the golden vectors, and size-independent properties at full size
(encode -> erase -> reconstruct round trips).  Reference call sites:
Encode main.go:262 (shardInput main.go:243-267), Decode main.go:77.
"""
import hashlib
import itertools
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)

import rsmi  # noqa: E402
from oracle import oracle  # noqa: E402

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "rs_golden.json")
_FECS = {}


def fec(k, n):
    if (k, n) not in _FECS:
        _FECS[(k, n)] = rsmi.NewFEC(k, n)
    return _FECS[(k, n)]


def collect(f, data):
    shares = [None] * f.Total()

    def out(s):
        shares[s.Number] = s.DeepCopy()  # main.go:255-258

    f.Encode(data, out)
    return shares


# ---------------------------------------------------------------- encode ----
CONFIGS = [(1, 1), (1, 2), (2, 3), (3, 5), (4, 6), (8, 14), (10, 14), (16, 20), (17, 49),
           (64, 80), (64, 100), (100, 120), (200, 256), (255, 256)]


@pytest.mark.parametrize("k,n", CONFIGS)
@pytest.mark.parametrize("S", [1, 15, 16, 17, 4099])
def test_encode_matches_oracle(k, n, S):
    f = fec(k, n)
    E = oracle.fec_matrix(k, n)
    assert f.matrix() == E.tobytes()
    data = oracle.splitmix_bytes(k * S, 31 * k + n + S).tobytes()
    shares = collect(f, data)
    for i in range(k):  # systematic: data shares are the input slices
        assert bytes(shares[i].Data) == data[i * S:(i + 1) * S]
    got = b"".join(bytes(shares[i].Data) for i in range(k, n))
    assert got == oracle.encode(E, k, n, data)


def test_encode_golden_vectors():
    with open(GOLDEN) as fh:
        g = json.load(fh)
    for rec in g["encodings"]:
        k, n, S = rec["k"], rec["n"], rec["S"]
        data = oracle.splitmix_bytes(k * S, rec["seed"]).tobytes()
        par = fec(k, n).encode_parity(data)
        assert hashlib.sha256(par).hexdigest() == rec["parity_sha256"], (k, n, S)


def test_encode_plugin_config1_blob():
    # BASELINE config 1: 1 MiB blob zero-padded to 1,048,580 B, RS(10,4).
    blob = oracle.splitmix_bytes(1 << 20, 0x5EED).tobytes() + b"\0" * 4
    f = fec(10, 14)
    assert f.encode_parity(blob) == oracle.encode(oracle.fec_matrix(10, 14), 10, 14, blob)


def test_encode_errors_and_empty():
    f = fec(4, 6)
    with pytest.raises(rsmi.RSError) as ei:
        f.Encode(b"abcde", lambda s: None)
    assert ei.value.code == rsmi.RS_ELEN_NOT_MULTIPLE
    got = collect(f, b"")
    assert all(len(s.Data) == 0 for s in got)


# ---------------------------------------------------------------- decode ----
def _shards(k, n, S, seed):
    data = oracle.splitmix_bytes(k * S, seed).tobytes()
    par = oracle.encode(oracle.fec_matrix(k, n), k, n, data)
    sh = [data[i * S:(i + 1) * S] for i in range(k)] + [par[i * S:(i + 1) * S] for i in range(n - k)]
    return data, sh


def test_decode_all_erasure_patterns_rs10_4():
    k, n, S = 10, 14, 100
    data, sh = _shards(k, n, S, 4242)
    f = fec(k, n)
    for e in range(0, n - k + 1):
        for lost in itertools.combinations(range(n), e):
            keep = [i for i in range(n) if i not in lost][-k:][::-1]
            shares = [rsmi.Share(i, sh[i]) for i in keep]
            assert f.Decode(None, shares) == data, lost
            assert [s.Number for s in shares] == sorted(keep)  # sorted in place


@pytest.mark.parametrize("k,n", [(4, 6), (8, 14), (17, 49), (64, 80), (200, 256)])
def test_decode_matches_oracle(k, n):
    rng = np.random.default_rng(k * 1000 + n)
    S = 333
    data, sh = _shards(k, n, S, k + n)
    f = fec(k, n)
    E = oracle.fec_matrix(k, n)
    for _ in range(4):
        keep = sorted(rng.choice(n, size=k, replace=False).tolist())
        rng.shuffle(keep)
        rc, ref = oracle.decode(E, k, n, [(i, sh[i]) for i in keep])
        assert rc == 0 and ref == data
        assert f.Decode(None, [rsmi.Share(i, sh[i]) for i in keep]) == ref


def test_decode_more_than_k_shares():
    k, n, S = 4, 6, 64
    data, sh = _shards(k, n, S, 5)
    assert fec(k, n).Decode(None, [rsmi.Share(i, sh[i]) for i in (5, 1, 4, 2, 3)]) == data


def test_decode_errors():
    k, n, S = 4, 6, 16
    data, sh = _shards(k, n, S, 6)
    f = fec(k, n)
    with pytest.raises(rsmi.NotEnoughShares):
        f.Decode(None, [rsmi.Share(i, sh[i]) for i in range(3)])
    with pytest.raises(rsmi.RSError) as ei:
        f.Decode(None, [rsmi.Share(i, sh[i]) for i in (0, 1, 2)] + [rsmi.Share(7, sh[3])])
    assert ei.value.code == rsmi.RS_EBAD_SHARE_ID
    with pytest.raises(rsmi.RSError) as ei:
        f.Decode(None, [rsmi.Share(i, sh[i]) for i in (0, 0, 1, 2)])
    assert ei.value.code == rsmi.RS_ESINGULAR
    with pytest.raises(rsmi.RSError) as ei:
        f.Decode(None, [rsmi.Share(0, sh[0]), rsmi.Share(1, sh[1][:5]), rsmi.Share(2, sh[2]),
                        rsmi.Share(3, sh[3])])
    assert ei.value.code == rsmi.RS_ESHARE_LEN


# ------------------------------------------------------- batched (device) ----
def _dev_stripes(f, stripes, S, pitch, seed):
    k, m = f.k, f.n - f.k
    data = torch.empty(stripes * k * pitch, dtype=torch.uint8, device="cuda")
    f.fill_splitmix(data.data_ptr(), data.numel(), seed)
    parity = torch.zeros(stripes * m * pitch, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    return data, parity


@pytest.mark.parametrize("k,n,S,pitch", [(10, 14, 65536, 65536), (10, 14, 1000, 1024),
                                         (4, 6, 4096, 4096), (64, 80, 65536, 65536),
                                         (17, 49, 4000, 4096), (8, 14, 100, 112)])
def test_encode_stripes_matches_oracle(k, n, S, pitch):
    f = fec(k, n)
    m = n - k
    stripes = 7
    data, parity = _dev_stripes(f, stripes, S, pitch, 77 + k)
    f.encode_stripes(data.data_ptr(), k * pitch, parity.data_ptr(), m * pitch, pitch, S, stripes)
    f.sync()
    hd = data.cpu().numpy().reshape(stripes, k, pitch)
    hp = parity.cpu().numpy().reshape(stripes, m, pitch)
    E = oracle.fec_matrix(k, n)
    for s in range(stripes):
        ref = oracle.encode(E, k, n, hd[s, :, :S].tobytes())
        assert hp[s, :, :S].tobytes() == ref, s


def _fec_with_env(k, n, bitslice):
    old = os.environ.get("RSMI_BITSLICE")
    os.environ["RSMI_BITSLICE"] = bitslice
    try:
        return rsmi.NewFEC(k, n)  # the kernel choice is made at rs_new
    finally:
        if old is None:
            del os.environ["RSMI_BITSLICE"]
        else:
            os.environ["RSMI_BITSLICE"] = old


def test_bitslice_kernel_selection():
    """The generated kernel serves RS(64,16) and RS(8,14) by default, RS(10,4)
    on request."""
    assert fec(64, 80).kernel_name(0) == "bitslice_k64_m16"
    assert fec(8, 14).kernel_name(0) == "bitslice_k8_m6"
    assert _fec_with_env(8, 14, "0").kernel_name(0).startswith("K8_MG6")
    assert fec(10, 14).kernel_name(0).startswith("K10_MG4")
    assert _fec_with_env(10, 14, "1").kernel_name(0) == "bitslice_k10_m4"
    assert _fec_with_env(64, 80, "0").kernel_name(0).startswith("K64_MG16")
    assert fec(17, 49).kernel_name(0).startswith("K0_")  # no generated kernel


@pytest.mark.parametrize("k,n", [(64, 80), (10, 14), (8, 14)])
@pytest.mark.parametrize("S,pitch", [(16, 16), (17, 32), (1000, 1008), (8192, 8192),
                                     (8192 + 16, 8208), (65536, 65536), (100000, 100000)])
def test_bitslice_encode_stripes_matches_oracle(k, n, S, pitch):
    """Generated bit-sliced encode (bitslice.hpp), bit-exact vs the oracle,
    ragged shard lengths (partial waves, a lone 16-B column, S % 16 != 0)."""
    f = _fec_with_env(k, n, "1")
    assert f.kernel_name(0).startswith("bitslice")
    m = n - k
    stripes = 3
    data, parity = _dev_stripes(f, stripes, S, pitch, 5 + S)
    f.encode_stripes(data.data_ptr(), k * pitch, parity.data_ptr(), m * pitch, pitch, S, stripes)
    f.sync()
    hd = data.cpu().numpy().reshape(stripes, k, pitch)
    hp = parity.cpu().numpy().reshape(stripes, m, pitch)
    E = oracle.fec_matrix(k, n)
    for s in range(stripes):
        assert hp[s, :, :S].tobytes() == oracle.encode(E, k, n, hd[s, :, :S].tobytes()), s
    f.close()


def test_bitslice_host_api_encode_matches_table_kernel():
    """rs_encode (pinned pipeline) through the generated kernel equals the
    split-table kernel and the oracle on a 4 MiB RS(64,16) message."""
    a, b = _fec_with_env(64, 80, "1"), _fec_with_env(64, 80, "0")
    data = oracle.splitmix_bytes(64 * 65536, 99).tobytes()
    pa, pb = collect(a, data), collect(b, data)
    assert all(bytes(x.Data) == bytes(y.Data) for x, y in zip(pa, pb))
    got = b"".join(bytes(pa[i].Data) for i in range(64, 80))
    assert got == oracle.encode(oracle.fec_matrix(64, 80), 64, 80, data)
    a.close()
    b.close()


def _fec_env(k, n, **env):
    """FEC built with RSMI_* knobs set (the kernel choice is made at rs_new)."""
    old = {key: os.environ.get(key) for key in env}
    os.environ.update(env)
    try:
        return rsmi.NewFEC(k, n)
    finally:
        for key, v in old.items():
            if v is None:
                del os.environ[key]
            else:
                os.environ[key] = v


def test_bitslice_reconstruct_kernel_selection():
    """Batched reconstruct of a bit-sliced code goes through the generated
    syndrome kernel (bitslice.hpp) unless RSMI_BITSLICE_REC=0."""
    assert fec(64, 80).kernel_name(1) == "bitslice_rec_k64_m16"
    assert _fec_env(64, 80, RSMI_BITSLICE_TOPS="1").kernel_name(1) == "bitslice_rec_k64_m16 +t4,8"
    assert _fec_env(64, 80, RSMI_BITSLICE_REC_MIN_E="5").kernel_name(1) == \
        "K64_MG4_B256 (e<5) + bitslice_rec_k64_m16"
    assert _fec_env(64, 80, RSMI_BITSLICE_REC="0").kernel_name(1).startswith("K64_MG16")
    assert fec(10, 14).kernel_name(1).startswith("K10_MG4")
    assert _fec_env(10, 14, RSMI_BITSLICE="1", RSMI_BITSLICE_REC_MIN_E="1").kernel_name(1) == \
        "bitslice_rec_k10_m4"
    assert fec(8, 14).kernel_name(1) == "bitslice_rec_k8_m6"
    assert _fec_env(8, 14, RSMI_BITSLICE="0").kernel_name(1).startswith("K8_MG")


def _fixed_patterns(k, n):
    """Edge erasure sets: every single erasure, all-data, all-parity, the
    m highest data shards, alternating, the first/last shard pairs, and sets
    straddling data shard 31/32 (the two words of the syndrome kernel's
    present-data mask: a set bit 31 of the low word once sign-extended over
    the high word, profiles/r03k/)."""
    m = n - k
    pats = [[i] for i in range(n)]
    if k > 33:
        pats += [[31, 32], [33, 40, k - 1], [30, 31, 32, 33][:m], [32, k][:m]]
    pats += [list(range(min(m, k))), list(range(k, n)), list(range(k - min(m, k), k)),
             list(range(0, n, 2))[:m], [0, n - 1], [k - 1, k]]
    out = np.zeros((len(pats), n), dtype=np.uint8)
    for r, p in enumerate(pats):
        out[r, p[:m]] = 1
    return out


@pytest.mark.parametrize("k,n", [(64, 80), (10, 14), (8, 14)])
@pytest.mark.parametrize("S,pitch", [(16, 16), (17, 32), (1000, 1008), (8192 + 16, 8208),
                                     (65536, 65536), (100000, 100000)])
def test_bitslice_reconstruct_roundtrip(k, n, S, pitch):
    """Generated bit-sliced reconstruct: random 1..m erasures plus the edge
    patterns, ragged shard lengths; regenerated shards equal the originals
    and the split-table kernel's output (both must be the unique codeword)."""
    m = n - k
    fb = _fec_env(k, n, RSMI_BITSLICE="1", RSMI_BITSLICE_REC_MIN_E="1")  # every stripe
    ft = _fec_env(k, n, RSMI_BITSLICE="0", RSMI_BITSLICE_REC="0")
    assert fb.kernel_name(1).startswith("bitslice_rec") and "bitslice" not in ft.kernel_name(1)
    rng = np.random.default_rng(k * 7 + S)
    er = np.concatenate([_fixed_patterns(k, n), _erasures(rng, 24, n, m)])
    stripes = len(er)
    data, parity = _dev_stripes(fb, stripes, S, pitch, 17 + S)
    fb.encode_stripes(data.data_ptr(), k * pitch, parity.data_ptr(), m * pitch, pitch, S, stripes)
    fb.sync()
    d0, p0 = data.clone(), parity.clone()
    for f in (fb, ft):
        data.copy_(d0)
        parity.copy_(p0)
        dv, pv = data.view(stripes, k, pitch), parity.view(stripes, m, pitch)
        dv[torch.from_numpy(er[:, :k].astype(bool)).cuda()] = 0xA5
        pv[torch.from_numpy(er[:, k:].astype(bool)).cuda()] = 0x5A
        f.reconstruct_stripes(data.data_ptr(), k * pitch, parity.data_ptr(), m * pitch, pitch, S,
                              stripes, er.tobytes())
        f.sync()
        dv0, pv0 = d0.view(stripes, k, pitch), p0.view(stripes, m, pitch)
        assert torch.equal(dv[:, :, :S], dv0[:, :, :S]), f.kernel_name(1)
        assert torch.equal(pv[:, :, :S], pv0[:, :, :S]), f.kernel_name(1)
    fb.close()
    ft.close()


_DIAG_CHILD = r"""
import sys
import numpy as np
import torch
root = sys.argv[1]
sys.path[:0] = [root, root + "/noise-erasurecode-plugin_amd"]
import rsmi
er = np.load(sys.argv[2])
k, n, S = 64, 80, 65536
m = n - k
f = rsmi.FEC(k, n)
assert f.kernel_name(1).startswith("bitslice_rec"), f.kernel_name(1)
stripes = len(er)
data = torch.empty(stripes * k * S, dtype=torch.uint8, device="cuda")
parity = torch.empty(stripes * m * S, dtype=torch.uint8, device="cuda")
f.fill_splitmix(data.data_ptr(), data.numel(), 99)
f.encode_stripes(data.data_ptr(), k * S, parity.data_ptr(), m * S, S, S, stripes)
f.sync()
d0, p0 = data.clone(), parity.clone()
data.view(stripes, k, S)[torch.from_numpy(er[:, :k].astype(bool)).cuda()] = 0
parity.view(stripes, m, S)[torch.from_numpy(er[:, k:].astype(bool)).cuda()] = 0
f.reconstruct_stripes(data.data_ptr(), k * S, parity.data_ptr(), m * S, S, S, stripes, er.tobytes())
f.sync()
assert torch.equal(data, d0) and torch.equal(parity, p0)
print("DIAG_DONE", flush=True)
"""


def test_mask_diagnostic_build(tmp_path):
    """the syndrome kernel clamps a parity survivor's slot
    (gen_bitslice.cpp) so that a wrong host mask record could only give wrong
    bytes, never a fault.  lib_diag/ (the Makefile's gen_bitslice -M build)
    re-derives every stripe's masks on the GPU from the pattern's id rows and
    prints RSMI_MASK_MISMATCH / RSMI_MASK_SLOT_OVERFLOW on any disagreement.
    Run it over the straddling edge sets and a fresh config-5 mix (1-16
    erasures, 512 stripes of 64 KiB): no report, and the round trip holds."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lib = os.path.join(root, "noise-erasurecode-plugin_amd", "lib_diag", "librsmi.so")
    assert os.path.exists(lib), "lib_diag/librsmi.so is built by `make diag` (build())"
    k, n = 64, 80
    er = np.concatenate([_fixed_patterns(k, n), _erasures(np.random.default_rng(16), 512, n, n - k)])
    np.save(tmp_path / "er.npy", er)
    env = dict(os.environ, RSMI_LIB=lib)
    r = subprocess.run([sys.executable, "-c", _DIAG_CHILD, root, str(tmp_path / "er.npy")], env=env,
                       capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "DIAG_DONE" in r.stdout, r.stdout[-2000:]
    assert "RSMI_MASK_" not in r.stdout, r.stdout[-2000:]


def _lowest_parity_row(er_row, k, n):
    """Python restatement of rsmi.cpp lowest_parity_row: the lowest parity
    row a pattern uses (erased parity outputs and Rebuild's parity
    survivors), m if none."""
    from rsmi import distributed as rd
    m = n - k
    used = [t for t in range(m) if er_row[k + t]]
    used += [i - k for i in rd.choose_survivors(er_row, k, n) if i >= k]
    return min(used) if used else m


@pytest.mark.parametrize("S,pitch", [(8192, 8192), (1000, 1008), (65536 + 16, 65536 + 16)])
def test_row_subset_syndrome_kernels(S, pitch):
    """with RSMI_BITSLICE_TOPS=1, RS(64,16) stripes whose
    patterns use only the top 4 or top 8 parity rows go to the row-subset
    syndrome kernels (t4: 101 VGPRs, t8: 135, vs 199 for all 16 rows; opt-in,
    measured no faster: profiles/r03i/).  Edge patterns on both sides of each
    boundary plus random ones, in one call (several launches); the result
    equals the originals and the default full kernel's."""
    k, n = 64, 80
    m = n - k
    pats = [
        [0], [63], [0, 1, 2, 3], [60, 61, 62, 63], [k + 15], [k + 12], [k + 12, 0, 1, 2],  # top 4
        [0, 1, 2, 3, 4], [k + 11], [k + 8, 5], list(range(8)), [k + 12, k + 13, 0, 1, 2, 3, 4, 5],  # top 8
        list(range(9)), [k + 7], [k + 0, 1], list(range(16)), list(range(k, n)),  # full
        [k + 15, k + 14, k + 13, k + 12, 0],  # 4 top rows erased + 1 data: survivor row 11 -> t8
    ]
    er = np.zeros((len(pats), n), dtype=np.uint8)
    for r, pl in enumerate(pats):
        er[r, pl] = 1
    rng = np.random.default_rng(S)
    er = np.concatenate([er, _erasures(rng, 40, n, m)])
    lows = [_lowest_parity_row(row, k, n) for row in er]
    assert {0, 1, 2} <= {0 if lo >= 12 else 1 if lo >= 8 else 2 for lo in lows}  # all three kernels used
    stripes = len(er)
    f_top = _fec_env(64, 80, RSMI_BITSLICE_TOPS="1")
    f_full = fec(64, 80)
    data, parity = _dev_stripes(f_top, stripes, S, pitch, 5 + S)
    f_top.encode_stripes(data.data_ptr(), k * pitch, parity.data_ptr(), m * pitch, pitch, S, stripes)
    f_top.sync()
    d0, p0 = data.clone(), parity.clone()
    for f in (f_top, f_full):
        data.copy_(d0)
        parity.copy_(p0)
        dv, pv = data.view(stripes, k, pitch), parity.view(stripes, m, pitch)
        dv[torch.from_numpy(er[:, :k].astype(bool)).cuda()] = 0xA5
        pv[torch.from_numpy(er[:, k:].astype(bool)).cuda()] = 0x5A
        f.reconstruct_stripes(data.data_ptr(), k * pitch, parity.data_ptr(), m * pitch, pitch, S, stripes,
                              er.tobytes())
        f.sync()
        dv0, pv0 = d0.view(stripes, k, pitch), p0.view(stripes, m, pitch)
        assert torch.equal(dv[:, :, :S], dv0[:, :, :S]), f.kernel_name(1)
        assert torch.equal(pv[:, :, :S], pv0[:, :, :S]), f.kernel_name(1)
    # and in pointer mode, every shard at a random row of a pool
    _check_ptrs_roundtrip(f_top, k, n, S, er, 77 + S)
    f_top.close()  # the env-built context; f_full is the shared cached one


def _check_ptrs_roundtrip(f, k, n, S, er, seed):
    stripes = len(er)
    Sp = (S + 15) // 16 * 16  # shard addresses must be 16-byte aligned
    pool = torch.empty((stripes * n, Sp), dtype=torch.uint8, device="cuda")
    f.fill_splitmix(pool.data_ptr(), pool.numel(), seed)
    rows = torch.from_numpy(np.random.default_rng(seed).permutation(stripes * n).reshape(stripes, n)).cuda()
    m = n - k
    data = torch.empty(stripes * k * Sp, dtype=torch.uint8, device="cuda")
    parity = torch.empty(stripes * m * Sp, dtype=torch.uint8, device="cuda")
    f.fill_splitmix(data.data_ptr(), data.numel(), seed + 1)
    f.encode_stripes(data.data_ptr(), k * Sp, parity.data_ptr(), m * Sp, Sp, S, stripes)
    f.sync()
    full = torch.cat([data.view(stripes, k, Sp), parity.view(stripes, m, Sp)], dim=1)[:, :, :S]
    pool[rows.view(-1), :S] = full.reshape(-1, S)
    erb = torch.from_numpy(er.astype(bool)).cuda()
    pool[rows[erb]] = 0
    table = (pool.data_ptr() + rows.to(torch.int64) * Sp).contiguous()
    f.reconstruct_ptrs(table.data_ptr(), S, stripes, er.tobytes())
    f.sync()
    assert torch.equal(pool[rows.view(-1), :S].view(stripes, n, S), full)


@pytest.mark.parametrize("small_split", ["0", "16"])
@pytest.mark.parametrize("k,n", [(8, 14), (64, 80)])
def test_bitslice_rec_past_2gib(k, n, small_split):
    """the syndrome kernel's buffer loads gave a present
    input a 0x7FFFFFFF-byte range, so every column at or past 2 GiB read as
    zeros while rs_reconstruct_* accept shards up to 2^28 columns.  One
    pointer-mode stripe of (2^31 + 8,232)-byte shards: survivor i is the
    window of one random buffer starting at byte 16*i (distinct bytes per
    survivor, one allocation), data shards 1 and 5 erased.  The outputs at
    sampled columns on both sides of 2 GiB and at the ragged end equal the
    oracle's Rebuild of the same k survivors at those columns (Rebuild is
    column-wise linear, so any bytes will do, codeword or not).  small_split
    "0" keeps the one-stripe call on the syndrome kernel (the one the range
    bug was in); "16" (the default) sends it to the split-table kernel."""
    f = _fec_env(k, n, RSMI_SMALL_SPLIT=small_split)
    assert f.kernel_name(1).startswith("bitslice_rec")
    m = n - k
    S = (1 << 31) + 8192 + 40
    Sp = (S + 15) // 16 * 16
    X = torch.empty(Sp + 16 * n, dtype=torch.uint8, device="cuda")
    f.fill_splitmix(X.data_ptr(), X.numel(), 4242)
    erased = [1, 5]
    outs = [torch.zeros(Sp, dtype=torch.uint8, device="cuda") for _ in erased]
    table = [X.data_ptr() + 16 * i for i in range(n)]
    for t, i in enumerate(erased):
        table[i] = outs[t].data_ptr()
    tab = torch.tensor(table, dtype=torch.int64, device="cuda")
    er = np.zeros((1, n), dtype=np.uint8)
    er[0, erased] = 1
    syn0 = f.stat(f.STAT_REC_STRIPES_SYNDROME)
    f.reconstruct_ptrs(tab.data_ptr(), S, 1, er.tobytes())
    f.sync()
    assert f.stat(f.STAT_REC_STRIPES_SYNDROME) - syn0 == (1 if small_split == "0" else 0)  # the kernel under test ran
    c2g = 1 << 27  # the column at 2 GiB
    cols = [0, 1, 511, 512, c2g - 513, c2g - 1, c2g, c2g + 1, c2g + 511, c2g + 512, Sp // 16 - 2, Sp // 16 - 1]
    idx = torch.tensor([16 * c + b for c in cols for b in range(16)], dtype=torch.int64, device="cuda")
    # Rebuild's survivors: the present data shards and, for the d erased
    # data slots, the d highest-numbered parity shards.
    surv = [i for i in range(k) if i not in erased] + list(range(n - 1, n - 1 - len(erased), -1))
    shares = [(i, X[16 * i:][idx].cpu().numpy().tobytes()) for i in surv]
    rc, ref = oracle.decode(oracle.fec_matrix(k, n), k, n, shares)
    assert rc == 0
    L = 16 * len(cols)
    for t, i in enumerate(erased):
        got = outs[t][idx].cpu().numpy().tobytes()
        want = ref[i * L:(i + 1) * L]
        # the ragged last column holds S % 16 = 8 real bytes; the rest is padding
        assert got[:L - 8] == want[:L - 8], (k, n, i)
    del X, outs
    f.close()


def test_reconstruct_split_between_kernels():
    """RS(64,16) reconstruct with RSMI_BITSLICE_REC_MIN_E=5: stripes with
    e < 5 go to the split-table kernel, the rest to the syndrome kernel, in
    one call (two launches)."""
    k, n, S = 64, 80, 8192
    m = n - k
    f = _fec_env(64, 80, RSMI_BITSLICE_REC_MIN_E="5")
    rng = np.random.default_rng(77)
    er = np.concatenate([_erasures(rng, 10, n, m, emin=1, emax=4),
                         _erasures(rng, 10, n, m, emin=5, emax=16)])
    er = er[rng.permutation(len(er))]
    stripes = len(er)
    data, parity = _dev_stripes(f, stripes, S, S, 91)
    f.encode_stripes(data.data_ptr(), k * S, parity.data_ptr(), m * S, S, S, stripes)
    f.sync()
    d0, p0 = data.clone(), parity.clone()
    data.view(stripes, k, S)[torch.from_numpy(er[:, :k].astype(bool)).cuda()] = 0
    parity.view(stripes, m, S)[torch.from_numpy(er[:, k:].astype(bool)).cuda()] = 0
    f.reconstruct_stripes(data.data_ptr(), k * S, parity.data_ptr(), m * S, S, S, stripes,
                          er.tobytes())
    f.sync()
    assert torch.equal(data, d0) and torch.equal(parity, p0)


def test_bitslice_reconstruct_matches_oracle_rebuild():
    """RS(64,16) through the syndrome kernel: the regenerated data shards are
    the oracle's Rebuild of the same survivors (byte for byte)."""
    k, n, S, stripes = 64, 80, 4096, 6
    m = n - k
    f = _fec_env(64, 80, RSMI_SMALL_SPLIT="0")  # 6 stripes: keep them on the syndrome kernel
    assert f.stat(f.STAT_REC_STRIPES_SYNDROME) == 0
    data, parity = _dev_stripes(f, stripes, S, S, 2024)
    f.encode_stripes(data.data_ptr(), k * S, parity.data_ptr(), m * S, S, S, stripes)
    f.sync()
    er = _erasures(np.random.default_rng(5), stripes, n, m, emin=m - 2, emax=m)
    hd = data.cpu().numpy().reshape(stripes, k, S).copy()
    hp = parity.cpu().numpy().reshape(stripes, m, S).copy()
    E = oracle.fec_matrix(k, n)
    data.view(stripes, k, S)[torch.from_numpy(er[:, :k].astype(bool)).cuda()] = 0
    parity.view(stripes, m, S)[torch.from_numpy(er[:, k:].astype(bool)).cuda()] = 0
    f.reconstruct_stripes(data.data_ptr(), k * S, parity.data_ptr(), m * S, S, S, stripes,
                          er.tobytes())
    f.sync()
    got = data.cpu().numpy().reshape(stripes, k, S)
    for s in range(stripes):
        sh = [hd[s, i].tobytes() for i in range(k)] + [hp[s, i].tobytes() for i in range(m)]
        keep = [i for i in range(n) if not er[s, i]]
        rc, ref = oracle.decode(E, k, n, [(i, sh[i]) for i in keep[:k]])
        assert rc == 0 and ref == got[s].tobytes(), s
    assert parity.cpu().numpy().reshape(stripes, m, S).tobytes() == hp.tobytes()
    assert f.stat(f.STAT_REC_STRIPES_SYNDROME) == stripes


def test_fill_splitmix_matches_oracle():
    f = fec(10, 14)
    for n_bytes in (1, 7, 8, 4099, 1 << 16):
        t = torch.empty(n_bytes + 8, dtype=torch.uint8, device="cuda")
        f.fill_splitmix(t.data_ptr(), n_bytes, 1234)
        f.sync()
        assert t[:n_bytes].cpu().numpy().tobytes() == oracle.splitmix_bytes(n_bytes, 1234).tobytes()


def _erasures(rng, stripes, n, m, emin=1, emax=None):
    emax = m if emax is None else emax
    er = np.zeros((stripes, n), dtype=np.uint8)
    for s in range(stripes):
        e = int(rng.integers(emin, emax + 1))
        er[s, rng.choice(n, size=e, replace=False)] = 1
    return er


@pytest.mark.parametrize("k,n,S,pitch,stripes", [(10, 14, 65536, 65536, 64),
                                                 (10, 14, 999, 1008, 50),
                                                 (4, 6, 4096, 4096, 40),
                                                 (64, 80, 65536, 65536, 6),
                                                 (17, 49, 4000, 4096, 9)])
def test_reconstruct_stripes_roundtrip(k, n, S, pitch, stripes):
    f = fec(k, n)
    m = n - k
    rng = np.random.default_rng(k + n + S)
    data, parity = _dev_stripes(f, stripes, S, pitch, 900 + k)
    f.encode_stripes(data.data_ptr(), k * pitch, parity.data_ptr(), m * pitch, pitch, S, stripes)
    f.sync()
    d0, p0 = data.clone(), parity.clone()
    er = _erasures(rng, stripes, n, m)
    dv = data.view(stripes, k, pitch)
    pv = parity.view(stripes, m, pitch)
    for s in range(stripes):  # destroy the erased shards
        for i in np.nonzero(er[s])[0]:
            (dv[s, i] if i < k else pv[s, i - k]).fill_(0xA5)
    f.reconstruct_stripes(data.data_ptr(), k * pitch, parity.data_ptr(), m * pitch, pitch, S,
                          stripes, er.tobytes())
    f.sync()
    dv0, pv0 = d0.view(stripes, k, pitch), p0.view(stripes, m, pitch)
    assert torch.equal(dv[:, :, :S], dv0[:, :, :S])
    assert torch.equal(pv[:, :, :S], pv0[:, :, :S])


def test_reconstruct_too_many_erasures_rejected():
    f = fec(4, 6)
    data, parity = _dev_stripes(f, 2, 256, 256, 1)
    er = np.zeros((2, 6), dtype=np.uint8)
    er[1, :3] = 1
    with pytest.raises(rsmi.NotEnoughShares):
        f.reconstruct_stripes(data.data_ptr(), 4 * 256, parity.data_ptr(), 2 * 256, 256, 256, 2,
                              er.tobytes())


def test_reconstruct_matches_oracle_rows():
    """Regenerated shards equal the oracle's Rebuild of the same survivors."""
    k, n, S, stripes = 10, 14, 4096, 12
    f = fec(k, n)
    m = n - k
    rng = np.random.default_rng(3)
    data, parity = _dev_stripes(f, stripes, S, S, 55)
    f.encode_stripes(data.data_ptr(), k * S, parity.data_ptr(), m * S, S, S, stripes)
    f.sync()
    er = _erasures(rng, stripes, n, m, emin=4, emax=4)
    hd = data.cpu().numpy().reshape(stripes, k, S)
    hp = parity.cpu().numpy().reshape(stripes, m, S)
    E = oracle.fec_matrix(k, n)
    for s in range(stripes):
        sh = [hd[s, i].tobytes() for i in range(k)] + [hp[s, i].tobytes() for i in range(m)]
        keep = [i for i in range(n) if not er[s, i]]
        rc, ref = oracle.decode(E, k, n, [(i, sh[i]) for i in keep[:k]])
        assert rc == 0 and ref == hd[s].tobytes()
    f.reconstruct_stripes(data.data_ptr(), k * S, parity.data_ptr(), m * S, S, S, stripes,
                          er.tobytes())
    f.sync()
    assert data.cpu().numpy().reshape(stripes, k, S).tobytes() == hd.tobytes()


def test_full_size_rs10_4_roundtrip():
    """BASELINE geometry (1 MiB shards), 256 stripes: encode, spot-check
    parity against the oracle, erase 1-4 shards per stripe, reconstruct,
    compare everything on the device."""
    k, n, S, stripes = 10, 14, 1 << 20, 256
    f = fec(k, n)
    m = n - k
    data, parity = _dev_stripes(f, stripes, S, S, 0x5EED)
    f.encode_stripes(data.data_ptr(), k * S, parity.data_ptr(), m * S, S, S, stripes)
    f.sync()
    E = oracle.fec_matrix(k, n)
    for s in (0, 131, 255):
        hd = data[s * k * S:(s + 1) * k * S].cpu().numpy().tobytes()
        hp = parity[s * m * S:(s + 1) * m * S].cpu().numpy().tobytes()
        assert hp == oracle.encode(E, k, n, hd)
    d0, p0 = data.clone(), parity.clone()
    er = _erasures(np.random.default_rng(0xE4A5), stripes, n, m)
    erd = torch.from_numpy(er[:, :k].astype(bool)).cuda()
    erp = torch.from_numpy(er[:, k:].astype(bool)).cuda()
    data.view(stripes, k, S)[erd] = 0
    parity.view(stripes, m, S)[erp] = 0
    f.reconstruct_stripes(data.data_ptr(), k * S, parity.data_ptr(), m * S, S, S, stripes,
                          er.tobytes())
    f.sync()
    assert torch.equal(data, d0)
    assert torch.equal(parity, p0)


def test_config2_full_size_64GiB_roundtrip():
    """The exact bench workload (BASELINE configs[1]+[2]): 6,553 RS(10,4)
    stripes x 10 x 1 MiB = 64 GiB of data + 25.6 GiB of parity, offsets far
    past 4 GiB.  Encode -> oracle spot checks of stripes whose bytes straddle
    or lie beyond the 32-bit boundary in both regions -> erase 1-4 random
    shards per stripe (bench.py's generator and seed) -> reconstruct ->
    torch.equal of all 89.6 GiB against a device clone, plus the oracle's
    Rebuild of the spot-checked stripes."""
    import bench
    k, n, S, stripes = 10, 14, 1 << 20, 6553
    m = n - k
    free, _ = torch.cuda.mem_get_info()
    need = 2 * stripes * n * S + (1 << 30)
    if free < need:
        pytest.skip(f"needs {need >> 30} GiB free on the device")
    f = fec(k, n)
    data = torch.empty(stripes * k * S, dtype=torch.uint8, device="cuda")
    parity = torch.empty(stripes * m * S, dtype=torch.uint8, device="cuda")
    f.fill_splitmix(data.data_ptr(), data.numel(), 0x5EED)
    f.fill_splitmix(parity.data_ptr(), parity.numel(), 1)
    f.encode_stripes(data.data_ptr(), k * S, parity.data_ptr(), m * S, S, S, stripes)
    f.sync()
    E = oracle.fec_matrix(k, n)
    # 409: data straddles 2^32; 1023/1024: parity around 2^32; 3276 and the
    # last stripe: data offsets ~34 GB and ~68.7 GB.
    spots = (0, 409, 1023, 1024, 3276, stripes - 1)
    assert 409 * k * S < (1 << 32) < 410 * k * S and 1024 * m * S == (1 << 32)
    host = {}
    for s in spots:
        hd = data[s * k * S:(s + 1) * k * S].cpu().numpy().tobytes()
        hp = parity[s * m * S:(s + 1) * m * S].cpu().numpy().tobytes()
        assert hp == oracle.encode(E, k, n, hd), s
        host[s] = [hd[i * S:(i + 1) * S] for i in range(k)] + [hp[i * S:(i + 1) * S] for i in range(m)]
    d0, p0 = data.clone(), parity.clone()
    rng = np.random.default_rng(0xE4A5)
    er = bench.erasure_sets(rng, 1, stripes, n, 1, m)[0]
    data.view(stripes, k, S)[torch.from_numpy(er[:, :k].astype(bool)).cuda()] = 0
    parity.view(stripes, m, S)[torch.from_numpy(er[:, k:].astype(bool)).cuda()] = 0
    f.prepare_patterns(m)
    f.reconstruct_stripes(data.data_ptr(), k * S, parity.data_ptr(), m * S, S, S, stripes,
                          er.tobytes())
    f.sync()
    for s in spots:  # regenerated bytes vs the oracle's Rebuild of the same survivors
        keep = [i for i in range(n) if not er[s, i]]
        rc, ref = oracle.decode(E, k, n, [(i, host[s][i]) for i in keep[:k]])
        assert rc == 0 and ref == data[s * k * S:(s + 1) * k * S].cpu().numpy().tobytes(), s
    assert torch.equal(data, d0)
    assert torch.equal(parity, p0)
    del data, parity, d0, p0
    torch.cuda.empty_cache()


def test_config5_full_size_roundtrip():
    """BASELINE configs[4] at the bench's size: 16,384 RS(64,16) stripes x
    80 x 64 KiB (64 GiB data + 16 GiB parity) through the bit-sliced encode
    and the syndrome reconstruct in their XCD-aware block order.  Encode ->
    oracle spot checks (first, middle, last stripe) -> erase 1-16 random
    shards per stripe (a fresh pattern almost every stripe) -> reconstruct ->
    torch.equal of all 80 GiB against a device clone."""
    import bench
    k, n, S, stripes = 64, 80, 1 << 16, 16384
    m = n - k
    free, _ = torch.cuda.mem_get_info()
    need = 2 * stripes * n * S + (1 << 30)
    if free < need:
        pytest.skip(f"needs {need >> 30} GiB free on the device")
    f = fec(k, n)
    assert f.kernel_name(0).startswith("bitslice") and f.kernel_name(1).startswith("bitslice_rec")
    data = torch.empty(stripes * k * S, dtype=torch.uint8, device="cuda")
    parity = torch.empty(stripes * m * S, dtype=torch.uint8, device="cuda")
    f.fill_splitmix(data.data_ptr(), data.numel(), 0xC5)
    f.fill_splitmix(parity.data_ptr(), parity.numel(), 2)
    f.encode_stripes(data.data_ptr(), k * S, parity.data_ptr(), m * S, S, S, stripes)
    f.sync()
    E = oracle.fec_matrix(k, n)
    for s in (0, stripes // 2 + 3, stripes - 1):
        hd = data[s * k * S:(s + 1) * k * S].cpu().numpy().tobytes()
        hp = parity[s * m * S:(s + 1) * m * S].cpu().numpy().tobytes()
        assert hp == oracle.encode(E, k, n, hd), s
    d0, p0 = data.clone(), parity.clone()
    rng = np.random.default_rng(0xE4A6)
    er = bench.erasure_sets(rng, 1, stripes, n, 1, m)[0]
    data.view(stripes, k, S)[torch.from_numpy(er[:, :k].astype(bool)).cuda()] = 0
    parity.view(stripes, m, S)[torch.from_numpy(er[:, k:].astype(bool)).cuda()] = 0
    f.reconstruct_stripes(data.data_ptr(), k * S, parity.data_ptr(), m * S, S, S, stripes,
                          er.tobytes())
    f.sync()
    assert torch.equal(data, d0)
    assert torch.equal(parity, p0)
    del data, parity, d0, p0
    torch.cuda.empty_cache()


@pytest.mark.parametrize("world", [1, 2, 3])
def test_distributed_gather_and_pointer_reconstruct(world):
    """rsmi.distributed end to end on one GPU: the holder buffers of `world`
    ranks, each rank's plan, the sender-side packing into the send buffer
    (what gather_survivors does before batch_isend_irecv), the transport
    emulated by copying every send segment into the matching receive segment,
    then rs_reconstruct_ptrs through each owner's shard table.  Outputs equal
    the originals.  (The RCCL transport itself: tests/test_distributed.py
    with gloo; world 1 calls gather_survivors, which moves nothing.)"""
    from rsmi import distributed as rd
    k, n, S, stripes = 10, 14, 4096, 19
    f = fec(k, n)
    data, parity = _dev_stripes(f, stripes, S, S, 31)
    f.encode_stripes(data.data_ptr(), k * S, parity.data_ptr(), (n - k) * S, S, S, stripes)
    f.sync()
    full = torch.cat([data.view(stripes, k, S), parity.view(stripes, n - k, S)], dim=1).contiguous()
    er = _erasures(np.random.default_rng(9 + world), stripes, n, n - k)
    held = [full[:, rd.local_shard_ids(r, n, world), :].contiguous() for r in range(world)]
    for chunks in (1, 3):
        plans = [rd.plan_exchange(er, k, n, r, world, S, chunks=chunks) for r in range(world)]
        bufs = [rd.make_buffers([plans[r]], S, "cuda") for r in range(world)]
        if world == 1:
            for c in range(len(plans[0].chunks)):
                rd.gather_survivors(held[0], plans[0], bufs[0], chunk=c)
        tables = [torch.from_numpy(rd.shard_table(plans[o], held[o], bufs[o])).cuda() for o in range(world)]
        for o in range(world):
            bufs[o].out.fill_(0xA5)
        for c in range(len(plans[0].chunks)):
            for p in range(world):  # sender packing of chunk c, as gather_survivors does it
                flat = held[p].view(-1, S)
                ch = plans[p].chunks[c]
                for o, rows in ch.send.items():
                    if len(rows):
                        seg = bufs[p].send[c % bufs[p].slots][ch.send_off[o]:ch.send_off[o] + len(rows)]
                        torch.index_select(flat, 0, torch.from_numpy(rows).cuda(), out=seg)
            for o in range(world):  # the transport into o's slot
                ch = plans[o].chunks[c]
                for p, cnt in ch.recv.items():
                    if cnt:
                        so = plans[p].chunks[c].send_off[o]
                        bufs[o].recv[c % bufs[o].slots][ch.recv_off[p]:ch.recv_off[p] + cnt].copy_(
                            bufs[p].send[c % bufs[p].slots][so:so + cnt])
            for o in range(world):  # chunk c's reconstruct (before its slot is reused)
                rd.reconstruct_owned(f, plans[o], tables[o], er[plans[o].owned], S, chunk=c)
            f.sync()
        for o in range(world):
            pl = plans[o]
            for j, s in enumerate(pl.owned):
                for i in np.nonzero(er[s])[0]:
                    assert torch.equal(bufs[o].out[int(pl.row[j, i])], full[s, i]), (world, chunks, o, s, i)


@pytest.mark.parametrize("k,n,S", [(10, 14, 4099), (64, 80, 8192), (4, 6, 100), (17, 49, 1000)])
def test_reconstruct_ptrs_scattered_shards(k, n, S):
    """rs_reconstruct_ptrs with every shard of every stripe at a random row of
    one pool (random order, shards of different stripes interleaved) equals
    the strided reconstruct: survivors read and erased shards written only
    through the table, for the split-table and the bit-sliced (RS(64,16))
    kernels."""
    f = fec(k, n)
    m = n - k
    stripes = 24
    pitch = (S + 15) // 16 * 16
    data, parity = _dev_stripes(f, stripes, S, pitch, 600 + k)
    f.encode_stripes(data.data_ptr(), k * pitch, parity.data_ptr(), m * pitch, pitch, S, stripes)
    f.sync()
    full = torch.cat([data.view(stripes, k, pitch), parity.view(stripes, m, pitch)], dim=1)
    rng = np.random.default_rng(k * 3 + S)
    er = _erasures(rng, stripes, n, m)
    perm = rng.permutation(stripes * n)
    pool = torch.empty((stripes * n, pitch), dtype=torch.uint8, device="cuda")
    pool[torch.from_numpy(perm).cuda()] = full.reshape(stripes * n, pitch)
    bad = torch.from_numpy(np.repeat(er.reshape(-1), 1).astype(bool))
    pool[torch.from_numpy(perm[bad.numpy()]).cuda()] = 0x3C  # erased rows destroyed
    table = torch.tensor((pool.data_ptr() + perm.astype(np.int64) * pitch).reshape(stripes, n),
                         dtype=torch.int64, device="cuda")
    f.reconstruct_ptrs(table.data_ptr(), S, stripes, er.tobytes())
    f.sync()
    got = pool[torch.from_numpy(perm).cuda()].view(stripes, n, pitch)
    assert torch.equal(got[:, :, :S], full[:, :, :S])


# ------------------------------------------------ GPU decode-row builder ----
def _host_rows(k, n, erased):
    """Rebuild's decode rows from the oracle: survivors by Rebuild's rule,
    inverse by the oracle's invertMatrix, rows = E[erased] . inverse."""
    import np_rs
    from rsmi import distributed as rd
    E = oracle.fec_matrix(k, n)
    surv = rd.choose_survivors(erased, k, n)
    rc, inv = oracle.invert(E[surv])
    assert rc == 0
    tg = [i for i in range(n) if erased[i]]
    return np_rs.matmul(E[tg], inv) if tg else np.zeros((0, k), np.uint8)


@pytest.mark.parametrize("k,n,count", [(10, 14, 0), (64, 80, 40), (17, 49, 30), (200, 256, 3), (100, 228, 4),
                                       (4, 6, 0)])
def test_gpu_inversion_matches_oracle(k, n, count):
    f = fec(k, n)
    m = n - k
    if count == 0:  # every pattern of <= m erasures
        pats = [c for e in range(1, m + 1) for c in itertools.combinations(range(n), e)]
    else:
        rng = np.random.default_rng(k + n)
        pats = [tuple(sorted(rng.choice(n, size=int(rng.integers(1, m + 1)), replace=False)))
                for _ in range(count)]
    for lost in pats:
        er = np.zeros(n, dtype=np.uint8)
        er[list(lost)] = 1
        rows, cnt = f.pattern_rows(er.tobytes())
        assert cnt == len(lost)
        got = np.frombuffer(rows, dtype=np.uint8).reshape(m, k)[:cnt]
        assert (got == _host_rows(k, n, er)).all(), lost


@pytest.mark.parametrize("k,n,count", [(10, 14, 0), (64, 80, 40), (17, 49, 30), (4, 6, 0)])
def test_gpu_inversion_generic_matches_oracle(k, n, count, monkeypatch):
    """The whole-matrix Gauss-Jordan path (RSMI_INVERT_GENERIC=1) gives the
    same rows as the structured d x d path and the oracle."""
    monkeypatch.setenv("RSMI_INVERT_GENERIC", "1")
    f = rsmi.FEC(k, n)  # fresh ctx: patterns built under the knob
    m = n - k
    if count == 0:
        pats = [c for e in range(1, m + 1) for c in itertools.combinations(range(n), e)]
    else:
        rng = np.random.default_rng(k * n)
        pats = [tuple(sorted(rng.choice(n, size=int(rng.integers(1, m + 1)), replace=False)))
                for _ in range(count)]
    for lost in pats:
        er = np.zeros(n, dtype=np.uint8)
        er[list(lost)] = 1
        rows, cnt = f.pattern_rows(er.tobytes())
        got = np.frombuffer(rows, dtype=np.uint8).reshape(m, k)[:cnt]
        assert (got == _host_rows(k, n, er)).all(), lost


def test_reconstruct_wide_code_unique_patterns():
    """RS(64,16), 64 KiB shards: every stripe has its own random 1-16-erasure
    pattern, so every decode matrix is built by the GPU inversion kernel."""
    k, n, S, stripes = 64, 80, 65536, 48
    f = rsmi.FEC(k, n)  # fresh ctx: empty pattern cache
    m = n - k
    data, parity = _dev_stripes(f, stripes, S, S, 4321)
    f.encode_stripes(data.data_ptr(), k * S, parity.data_ptr(), m * S, S, S, stripes)
    f.sync()
    d0, p0 = data.clone(), parity.clone()
    er = _erasures(np.random.default_rng(64), stripes, n, m)
    data.view(stripes, k, S)[torch.from_numpy(er[:, :k].astype(bool)).cuda()] = 0
    parity.view(stripes, m, S)[torch.from_numpy(er[:, k:].astype(bool)).cuda()] = 0
    f.reconstruct_stripes(data.data_ptr(), k * S, parity.data_ptr(), m * S, S, S, stripes,
                          er.tobytes())
    f.sync()
    assert f.pattern_count() == len({r.tobytes() for r in er})
    assert torch.equal(data, d0) and torch.equal(parity, p0)


# --------------------------------------- Decode with Correct (> k shares) ----
def _corrupt(sh, ids, rng, cols=None):
    out = [bytearray(x) for x in sh]
    for i in ids:
        if cols is None:
            out[i] = bytearray(rng.integers(0, 256, len(out[i]), dtype=np.uint8).tobytes())
        else:
            for c in cols:
                out[i][c] ^= int(rng.integers(1, 256))
    return [bytes(x) for x in out]


@pytest.mark.parametrize("k,n,bad", [(10, 14, [3]), (10, 14, [12]), (10, 14, [0, 13]),
                                     (4, 6, [1]), (64, 80, [0, 5, 17, 63, 64, 70, 71, 79])])
def test_decode_corrects_whole_share_errors(k, n, bad):
    S = 777
    data, sh = _shards(k, n, S, k * 7 + n)
    rng = np.random.default_rng(len(bad))
    cor = _corrupt(sh, bad, rng)
    shares = [rsmi.Share(i, cor[i]) for i in range(n)][::-1]
    assert fec(k, n).Decode(None, shares) == data
    rc, ref = oracle.decode_correct(oracle.fec_matrix(k, n), k, n, [(i, cor[i]) for i in range(n)])
    assert rc == 0 and ref == data


def test_decode_corrects_scattered_column_errors():
    """Different shares are bad in different columns (each column within the
    correction radius): the located-erasure pass leaves columns that need
    per-column Berlekamp-Welch."""
    k, n, S = 10, 14, 4096
    data, sh = _shards(k, n, S, 99)
    rng = np.random.default_rng(5)
    cor = [bytearray(x) for x in sh]
    for c in range(0, S, 7):
        for i in rng.choice(n, size=int(rng.integers(1, 3)), replace=False):
            cor[i][c] ^= int(rng.integers(1, 256))
    cor = [bytes(x) for x in cor]
    assert fec(k, n).Decode(None, [rsmi.Share(i, cor[i]) for i in range(n)]) == data
    rc, ref = oracle.decode_correct(oracle.fec_matrix(k, n), k, n, [(i, cor[i]) for i in range(n)])
    assert rc == 0 and ref == data


def test_decode_correct_error_cases():
    k, n, S = 10, 14, 256
    data, sh = _shards(k, n, S, 123)
    rng = np.random.default_rng(8)
    f = fec(k, n)
    cor = _corrupt(sh, [1, 6, 11], rng)  # 3 bad > floor(4/2)
    with pytest.raises(rsmi.RSError) as ei:
        f.Decode(None, [rsmi.Share(i, cor[i]) for i in range(n)])
    assert ei.value.code == rsmi.RS_ETOO_MANY_ERRORS
    rc, _ = oracle.decode_correct(oracle.fec_matrix(k, n), k, n, [(i, cor[i]) for i in range(n)])
    assert rc == -7
    cor = _corrupt(sh, [2], rng)  # k+1 shares: inconsistency found, nothing to correct with
    with pytest.raises(rsmi.NotEnoughShares):
        f.Decode(None, [rsmi.Share(i, cor[i]) for i in range(k + 1)])
    # exactly k shares: no check, like infectious (the corruption passes)
    got = f.Decode(None, [rsmi.Share(i, cor[i]) for i in range(k)])
    assert got != data and got[2 * S:3 * S] == cor[2]


# ------------------------------------ host API with pinned caller buffers ----
@pytest.mark.parametrize("k,n,S", [(10, 14, 104858), (4, 6, 17), (64, 80, 65536 + 16)])
def test_host_api_pinned_buffers(k, n, S):
    """The host-buffer API on caller buffers from rs_pinned_alloc (and a
    pinned source with a pageable destination): the same parity and decoded
    bytes as the oracle.  (A DMA-in-place path for pinned callers measured no
    faster than the staging pipeline -- pointer queries and per-shard copies
    cost what the staging copies did -- so all callers take that pipeline.)"""
    import ctypes
    lib = rsmi.load()
    f = fec(k, n)
    m = n - k
    E = oracle.fec_matrix(k, n)
    data = oracle.splitmix_bytes(k * S, k * 1000 + n).tobytes()
    ref = oracle.encode(E, k, n, data)
    pin_in = lib.rs_pinned_alloc(k * S)
    pin_par = lib.rs_pinned_alloc(m * S)
    pin_dst = lib.rs_pinned_alloc(k * S)
    assert pin_in and pin_par and pin_dst
    try:
        ctypes.memmove(pin_in, data, k * S)
        assert lib.rs_encode(f.handle, pin_in, k * S, pin_par) == rsmi.RS_OK
        assert ctypes.string_at(pin_par, m * S) == ref
        pageable = ctypes.create_string_buffer(m * S)
        assert lib.rs_encode(f.handle, pin_in, k * S, ctypes.cast(pageable, ctypes.c_void_p)) == rsmi.RS_OK
        assert pageable.raw == ref
        # decode from pinned shares: lose the first m data shares
        keep = list(range(m, k)) + list(range(k, n))
        shares = [pin_in + i * S if i < k else pin_par + (i - k) * S for i in keep][:k]
        nums = (ctypes.c_int * k)(*keep[:k])
        ptrs = (ctypes.c_void_p * k)(*shares)
        assert lib.rs_decode(f.handle, nums, ptrs, k, S, pin_dst) == rsmi.RS_OK
        assert ctypes.string_at(pin_dst, k * S) == data
    finally:
        for p in (pin_in, pin_par, pin_dst):
            lib.rs_pinned_free(p)


# Where each kept share sits relative to dst (rows of S bytes; dst row r is
# buffer row r + 1, so row -1 is just before dst).  Lost: data shares 0-3.
_ALIAS_LAYOUTS = {
    # share i one row after its own: copying share i to row i overwrites i - 1
    "plus1": lambda keep, k: {i: i + 1 for i in keep},
    # one row before its own: share i is overwritten by share i + 1's copy
    # before it is read
    "minus1": lambda keep, k: {i: i - 1 for i in keep},
    # Rebuild's parity survivors stored in the missing data rows the kernel
    # writes; present data shares in their own rows
    "missing_rows": lambda keep, k: {i: (i if i < k else i - k) for i in keep},
    # every share in dst, in reverse order
    "reversed": lambda keep, k: {i: k - 1 - j for j, i in enumerate(keep)},
}


@pytest.mark.parametrize("layout", sorted(_ALIAS_LAYOUTS))
@pytest.mark.parametrize("pinned", [True, False])
@pytest.mark.parametrize("S", [4096, 104858, 300000])
def test_decode_dst_overlapping_survivors(pinned, S, layout):
    """infectious lets Decode's shares alias dst.  rs_decode writes dst while
    the GPU still reads survivors -- in place when they are engine-pinned --
    and moves present shares within dst; the engine sets aliasing shares aside
    first.  Every layout decodes to the original data
    (engine-pinned and pageable memory; staged, chunked and pipelined sizes)."""
    import ctypes
    lib = rsmi.load()
    k, n = 10, 14
    f = fec(k, n)
    data, sh = _shards(k, n, S, 4321 + S)
    size = (n + 2) * S
    buf = lib.rs_pinned_alloc(size) if pinned else None
    keep_alive = None
    if not pinned:
        keep_alive = ctypes.create_string_buffer(size)
        buf = ctypes.addressof(keep_alive)
    assert buf
    try:
        lost = [0, 1, 2, 3]
        keep = [i for i in range(n) if i not in lost]
        row = _ALIAS_LAYOUTS[layout](keep, k)
        for i in keep:
            ctypes.memmove(buf + (row[i] + 1) * S, sh[i], S)
        nums = (ctypes.c_int * k)(*keep)
        ptrs = (ctypes.c_void_p * k)(*[buf + (row[i] + 1) * S for i in keep])
        assert lib.rs_decode(f.handle, nums, ptrs, k, S, buf + S) == rsmi.RS_OK
        assert ctypes.string_at(buf + S, k * S) == data
    finally:
        if pinned:
            lib.rs_pinned_free(buf)


@pytest.mark.parametrize("S,pitch", [(100, 112), (65536, 65536), (4099, 4112)])
def test_rs8_14_row_group_of_six(S, pitch):
    """RS(8,14) (infectious's example code) encodes with a 6-row group
    (K8_MG6: the last 4-row sub-step codes 2 rows) and reconstructs <= 4
    erasures with K8_MG4: parity vs the oracle, round trip vs the originals.
    The split-table kernels are forced (RSMI_BITSLICE=0): by default this
    code is bit-sliced (test_bitslice_*)."""
    k, n = 8, 14
    m = n - k
    f = _fec_with_env(k, n, "0")
    assert f.kernel_name(0).startswith("K8_MG6")
    stripes = 9
    data, parity = _dev_stripes(f, stripes, S, pitch, 88 + S)
    f.encode_stripes(data.data_ptr(), k * pitch, parity.data_ptr(), m * pitch, pitch, S, stripes)
    f.sync()
    hd = data.cpu().numpy().reshape(stripes, k, pitch)
    hp = parity.cpu().numpy().reshape(stripes, m, pitch)
    E = oracle.fec_matrix(k, n)
    for s in range(stripes):
        assert hp[s, :, :S].tobytes() == oracle.encode(E, k, n, hd[s, :, :S].tobytes()), s
    d0, p0 = data.clone(), parity.clone()
    for emax in (4, 6):  # K8_MG4 for <= 4 outputs, K8_MG6 beyond
        er = _erasures(np.random.default_rng(S + emax), stripes, n, m, emin=1, emax=emax)
        data.copy_(d0)
        parity.copy_(p0)
        data.view(stripes, k, pitch)[torch.from_numpy(er[:, :k].astype(bool)).cuda()] = 0
        parity.view(stripes, m, pitch)[torch.from_numpy(er[:, k:].astype(bool)).cuda()] = 0
        f.reconstruct_stripes(data.data_ptr(), k * pitch, parity.data_ptr(), m * pitch, pitch, S, stripes,
                              er.tobytes())
        f.sync()
        assert torch.equal(data.view(stripes, k, pitch)[:, :, :S], d0.view(stripes, k, pitch)[:, :, :S])
        assert torch.equal(parity.view(stripes, m, pitch)[:, :, :S], p0.view(stripes, m, pitch)[:, :, :S])


@pytest.mark.parametrize("k,n,env", [(10, 14, {}), (64, 80, {}), (64, 80, {"RSMI_SMALL_SPLIT": "0"}),
                                     (64, 80, {"RSMI_BITSLICE_REC_MIN_E": "5", "RSMI_SMALL_SPLIT": "0"}),
                                     (8, 14, {}), (8, 14, {"RSMI_SMALL_SPLIT": "0"})])
@pytest.mark.parametrize("stripes", [1, 2, 15, 16, 17, 40])
def test_inline_descriptor_threshold(k, n, env, stripes):
    """a reconstruct of at most 16 erased stripes passes its
    stripe descriptors (and mask records) in the kernel arguments instead of
    uploading them; more stripes upload.  Both sides of the threshold, every
    kernel (split table, syndrome, the two split between kernels in one
    call; a bit-sliced code's small calls go to the split table unless
    RSMI_SMALL_SPLIT=0), strided and pointer mode: the regenerated shards
    equal the originals and the upload path's output (RSMI_NO_INLINE_DESC)."""
    m = n - k
    S = 4096 + 48
    f_in = _fec_env(k, n, **env)
    f_up = _fec_env(k, n, RSMI_NO_INLINE_DESC="1", **env)
    rng = np.random.default_rng(stripes * 31 + k)
    er = _erasures(rng, stripes, n, m)
    if stripes > 2:
        er[1] = 0  # a stripe with nothing erased is skipped (not a descriptor)
    data, parity = _dev_stripes(f_in, stripes, S, S, 5 + stripes)
    f_in.encode_stripes(data.data_ptr(), k * S, parity.data_ptr(), m * S, S, S, stripes)
    f_in.sync()
    d0, p0 = data.clone(), parity.clone()
    erased = int((er.sum(axis=1) > 0).sum())
    bitsliced = "bitslice_rec" in f_in.kernel_name(1)
    small = env.get("RSMI_SMALL_SPLIT", "16") != "0" and erased <= 16
    for f in (f_in, f_up):
        data.copy_(d0)
        parity.copy_(p0)
        data.view(stripes, k, S)[torch.from_numpy(er[:, :k].astype(bool)).cuda()] = 0xEE
        parity.view(stripes, m, S)[torch.from_numpy(er[:, k:].astype(bool)).cuda()] = 0xEE
        t0, s0 = f.stat(f.STAT_REC_STRIPES_TABLE), f.stat(f.STAT_REC_STRIPES_SYNDROME)
        f.reconstruct_stripes(data.data_ptr(), k * S, parity.data_ptr(), m * S, S, S, stripes, er.tobytes())
        f.sync()
        assert torch.equal(data, d0) and torch.equal(parity, p0)
        dt, ds = f.stat(f.STAT_REC_STRIPES_TABLE) - t0, f.stat(f.STAT_REC_STRIPES_SYNDROME) - s0
        assert dt + ds == erased
        if not bitsliced or small:
            assert ds == 0, (dt, ds)  # the split-table kernel took every stripe
        elif "RSMI_BITSLICE_REC_MIN_E" not in env:
            assert dt == 0, (dt, ds)  # the syndrome kernel took every stripe
    _check_ptrs_roundtrip(f_in, k, n, S, er, 9 + stripes)
    f_in.close()
    f_up.close()


@pytest.mark.parametrize("k,n", [(10, 14), (64, 80), (200, 256)])
def test_erasure_flags_any_nonzero_byte(k, n):
    """rs_reconstruct_stripes treats any non-zero flag byte as erased (the
    pattern key is built 8 flags at a time, csrc/pattern_index.cpp): flags of
    0x80 / 0xFF / 0x01 mixed give the same bytes and the same patterns as
    flags of 1, on shards spanning every key word for n = 256."""
    f = fec(k, n)
    m = n - k
    stripes, S = 12, 4096
    data, parity = _dev_stripes(f, stripes, S, S, 900 + n)
    f.encode_stripes(data.data_ptr(), k * S, parity.data_ptr(), m * S, S, S, stripes)
    f.sync()
    d0, p0 = data.clone(), parity.clone()
    rng = np.random.default_rng(n)
    er = np.zeros((stripes, n), dtype=np.uint8)
    for s in range(stripes):
        er[s, rng.choice(n, size=int(rng.integers(1, m + 1)), replace=False)] = 1
    odd = er * rng.choice(np.array([0x01, 0x80, 0xFF, 0x10], dtype=np.uint8), size=er.shape)
    dv, pv = data.view(stripes, k, S), parity.view(stripes, m, S)
    for flags in (er, odd):
        for s in range(stripes):  # wipe the erased shards
            for i in np.nonzero(er[s])[0]:
                (dv[s, i] if i < k else pv[s, i - k]).fill_(0x5A)
        before = f.pattern_count()
        f.reconstruct_stripes(data.data_ptr(), k * S, parity.data_ptr(), m * S, S, S, stripes, flags.tobytes())
        f.sync()
        assert torch.equal(data, d0) and torch.equal(parity, p0)
        if flags is odd:
            assert f.pattern_count() == before  # same keys as the 0/1 flags


def test_pattern_tables_grow_across_calls():
    """A fresh random pattern for every stripe, call after call: the pattern
    tables grow x4 several times (outgrown buffers retired, no device sync)
    and every call's output stays exact.  RS(64,16), 16,384 stripes of
    256-byte shards, 13 calls -> ~213k patterns."""
    f = rsmi.FEC(64, 80)
    k, m, n = 64, 16, 80
    stripes, S = 16384, 256
    data, parity = _dev_stripes(f, stripes, S, S, 4242)
    f.encode_stripes(data.data_ptr(), k * S, parity.data_ptr(), m * S, S, S, stripes)
    f.sync()
    d0, p0 = data.clone(), parity.clone()
    rng = np.random.default_rng(77)
    for call in range(13):
        er = np.zeros((stripes, n), dtype=np.uint8)
        e = rng.integers(1, m + 1, size=stripes)
        for s in range(stripes):
            er[s, rng.choice(n, size=int(e[s]), replace=False)] = 1
        data.copy_(d0)
        parity.copy_(p0)
        mask = torch.from_numpy(er).to("cuda").bool()
        data.view(stripes, k, S)[mask[:, :k]] = 0
        parity.view(stripes, m, S)[mask[:, k:]] = 0
        f.reconstruct_stripes(data.data_ptr(), k * S, parity.data_ptr(), m * S, S, S, stripes, er.tobytes())
        f.sync()
        assert torch.equal(data, d0) and torch.equal(parity, p0), call
    assert f.pattern_count() > 150000 and f.pattern_evictions() == 0
    f.close()


@pytest.mark.gpu
@pytest.mark.parametrize("k,n,S", [(10, 14, 65536), (64, 80, 65536), (8, 14, 4096 + 48)])
@pytest.mark.parametrize("stripes", [1, 7, 8, 9, 17, 64])
def test_xcd_block_order_matches_natural(k, n, S, stripes):
    """The XCD-aware block order (csrc/xcd.hpp) only renumbers blocks: for
    stripe counts below, at and past multiples of 8 (the tail keeps the
    natural order) encode and 1..m-erasure reconstruct give the same bytes
    as the natural order (RSMI_XCD=0) and as the oracle, with the order
    forced on every kernel (RSMI_XCD=1) and with a region of 3 blocks for
    the split-table encode."""
    m = n - k
    # RSMI_SMALL_SPLIT=0: small calls stay on the bit-sliced kernels (whose block order is under test)
    fx = {"0": _fec_env(k, n, RSMI_XCD="0", RSMI_SMALL_SPLIT="0"), "1": _fec_env(k, n, RSMI_XCD="1", RSMI_SMALL_SPLIT="0"),
          "r3": _fec_env(k, n, RSMI_XCD_ENC_REGION="3", RSMI_SMALL_SPLIT="0")}
    rng = np.random.default_rng(stripes * 31 + k)
    er = _erasures(rng, stripes, n, m)
    data, parity = _dev_stripes(fx["0"], stripes, S, S, 5 + stripes)
    E = oracle.fec_matrix(k, n)
    hd = data.cpu().numpy()
    want = [oracle.encode(E, k, n, hd[s * k * S:(s + 1) * k * S].tobytes()) for s in range(stripes)]
    d0 = data.clone()
    for name, f in fx.items():
        parity.zero_()
        f.encode_stripes(data.data_ptr(), k * S, parity.data_ptr(), m * S, S, S, stripes)
        f.sync()
        hp = parity.cpu().numpy()
        for s in range(stripes):
            assert hp[s * m * S:(s + 1) * m * S].tobytes() == want[s], (name, s)
        p0 = parity.clone()
        dv, pv = data.view(stripes, k, S), parity.view(stripes, m, S)
        dv[torch.from_numpy(er[:, :k].astype(bool)).cuda()] = 0xA5
        pv[torch.from_numpy(er[:, k:].astype(bool)).cuda()] = 0x5A
        s0 = f.stat(f.STAT_REC_STRIPES_SYNDROME)
        f.reconstruct_stripes(data.data_ptr(), k * S, parity.data_ptr(), m * S, S, S, stripes, er.tobytes())
        f.sync()
        assert torch.equal(data, d0) and torch.equal(parity, p0), name
        if f.kernel_name(1).startswith("bitslice_rec"):
            assert f.stat(f.STAT_REC_STRIPES_SYNDROME) - s0 == int((er.sum(axis=1) > 0).sum()), name
    for f in fx.values():
        f.close()


@pytest.mark.parametrize("S", [1, 17, 8_200, 65_539, 209_700, 209_716, 209_733, 2 * 1024 * 1024 + 5])
@pytest.mark.parametrize("stage_small", [True, False])
def test_host_api_staging_threshold(S, stage_small, monkeypatch):
    """rs_encode / rs_decode on pageable buffers around the one-shot staging
    threshold (k x round_up(S, 16) <= 2 MiB: staged once and coded by one
    launch, rsmi.cpp encode_staged / decode_staged) and past it (the chunked
    pipeline, several 8 MiB chunks at S = 2 MiB + 5), unaligned shard
    lengths included, from one byte (one chunk below 8 KiB per shard, two
    column chunks from 256 KiB a message); RSMI_NO_STAGE_SMALL forces the
    pipeline for the small sizes too.  Bit-exact vs the oracle; decode with 4
    drops including parity, and with only parity lost (no launch: the
    present shares are copied)."""
    import ctypes
    if not stage_small:
        monkeypatch.setenv("RSMI_NO_STAGE_SMALL", "1")
    k, n = 10, 14
    m = n - k
    f = fec(k, n)
    lib = rsmi.load()
    E = oracle.fec_matrix(k, n)
    data = oracle.splitmix_bytes(k * S, S + 17)
    par = np.zeros(m * S, dtype=np.uint8)
    P = ctypes.c_void_p
    assert lib.rs_encode(f.handle, P(data.ctypes.data), k * S, P(par.ctypes.data)) == 0
    assert par.tobytes() == oracle.encode(E, k, n, data.tobytes())
    shard = lambda i: data[i * S:(i + 1) * S] if i < k else par[(i - k) * S:(i - k + 1) * S]
    for lost in ((0, 3, 7, 12), (1, 2, 10, 11), (9, 10, 11, 13), (10, 11, 12, 13)):
        keep = [i for i in range(n) if i not in lost]
        bufs = [np.ascontiguousarray(shard(i)) for i in keep]
        dst = np.zeros(k * S, dtype=np.uint8)
        nums = (ctypes.c_int * k)(*keep[::-1])
        ptrs = (ctypes.c_void_p * k)(*[b.ctypes.data for b in bufs[::-1]])
        assert lib.rs_decode(f.handle, nums, ptrs, k, S, P(dst.ctypes.data)) == 0
        assert np.array_equal(dst, data), lost


_CHUNKS_CHILD = r"""
import ctypes, os, sys
import numpy as np
sys.path[:0] = [os.environ["ROOT"], os.path.join(os.environ["ROOT"], "noise-erasurecode-plugin_amd")]
import rsmi
from oracle import oracle
k, n = 10, 14
m = n - k
f = rsmi.NewFEC(k, n)
lib = rsmi.load()
E = oracle.fec_matrix(k, n)
P = ctypes.c_void_p
for S in (8_193, 30_001, 104_858, 209_700):
    data = oracle.splitmix_bytes(k * S, S)
    par = np.zeros(m * S, dtype=np.uint8)
    assert lib.rs_encode(f.handle, P(data.ctypes.data), k * S, P(par.ctypes.data)) == 0
    assert par.tobytes() == oracle.encode(E, k, n, data.tobytes()), S
    shard = lambda i: data[i * S:(i + 1) * S] if i < k else par[(i - k) * S:(i - k + 1) * S]
    for lost in ((0, 3, 7, 12), (9, 10, 11, 13)):
        keep = [i for i in range(n) if i not in lost]
        bufs = [np.ascontiguousarray(shard(i)) for i in keep]
        dst = np.zeros(k * S, dtype=np.uint8)
        nums = (ctypes.c_int * k)(*keep)
        ptrs = (ctypes.c_void_p * k)(*[b.ctypes.data for b in bufs])
        assert lib.rs_decode(f.handle, nums, ptrs, k, S, P(dst.ctypes.data)) == 0
        assert np.array_equal(dst, data), (S, lost)
print("ok")
"""


@pytest.mark.parametrize("chunks", ["1", "3", "4"])
def test_host_api_forced_stage_chunks(chunks):
    """Staged small messages coded in 1, 3 or 4 column chunks
    (RSMI_STAGE_CHUNKS, read once per process: a child process each; the
    default 2 is covered above): each chunk is staged, launched and copied out
    on its own, chunk offsets 16-byte aligned, the last chunk ragged.
    Bit-exact vs the oracle."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, RSMI_STAGE_CHUNKS=chunks, ROOT=root)
    p = subprocess.run([sys.executable, "-c", _CHUNKS_CHILD], env=env, stdout=subprocess.PIPE,
                       stderr=subprocess.PIPE, text=True, timeout=120)
    assert p.returncode == 0 and p.stdout.strip() == "ok", p.stderr[-3000:]
