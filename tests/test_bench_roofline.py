"""bench.py's roofline bookkeeping for the configs[3] legs (CPU only): the
algorithmic bytes the resolution claim kernel is charged per candidate in
each table form (csrc/resolution.hip: packed one-word keys up to 31
variables, clause indices beyond), and which kernel the roofline names."""
import bench


def _stats(claim_ms, pair_ms):
    return [{"candidates": 1000, "pairs": 5000, "claim_ms": claim_ms, "pair_ms": pair_ms}] * 2


def test_claim_kernel_bytes_per_candidate():
    packed = bench.saturation_roofline(_stats(2.0, 1.0), nvars=12)
    index = bench.saturation_roofline(_stats(2.0, 1.0), nvars=40)
    assert packed["kernel"].startswith("ht_cand_packed_kernel")
    assert index["kernel"].startswith("ht_cand_kernel")
    # K = 2 words: key 16 B + slot read/CAS 16 B + flag 8 B; index form adds the
    # occupant key 16 B and the slot 8 B
    assert packed["algorithmic_bytes_per_step"] == 1000 * 40
    assert index["algorithmic_bytes_per_step"] == 1000 * 64
    assert abs(packed["achieved"] - 40e3 / 2e-3 / 1e9) < 1e-12
    assert packed["frac"] == packed["achieved"] / bench.HBM_PEAK_GBS


def test_pair_kernel_named_when_it_dominates():
    r = bench.saturation_roofline(_stats(0.5, 1.5), nvars=12)
    assert r["kernel"] == "res_pairs_kernel"
    assert r["algorithmic_bytes_per_step"] == 5000 * 16 + 1000 * 16
    assert bench.saturation_roofline([], nvars=12) is None
