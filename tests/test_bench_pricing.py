"""CPU: bench.py's algorithmic op pricing of the ML-KEM launches, which `roofline.achieved` divides
by the live launch durations.  Since round 4 the big launches are multi-role (mlkem.hip k_multi):
their ops are the sum of their roles', each counted as often per step as that launch runs."""
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "quantum-resistant-p2p_amd"))

bench = pytest.importorskip("bench")
PERM = 4320


@pytest.mark.parametrize("alg,k", [("ML-KEM-512", 2), ("ML-KEM-768", 3), ("ML-KEM-1024", 4)])
def test_multi_role_launches_count_each_role_once_per_launch(alg, k):
    ops = lambda name, mode="encdec": bench.kernel_ops_per_hs(alg, name, mode)[0]  # noqa: E731
    xof = 3 * k * k * PERM  # one SampleNTT pass
    assert ops("k_xof") == 2 * xof  # the stand-alone name: Encaps' and Decaps' passes
    # Encaps-only and Decaps-only launches run once per step, so their SampleNTT counts once
    assert ops("k_front_encaps+k_xof") == ops("k_front_encaps") + xof
    assert ops("k_j_decaps+k_decrypt_core+k_xof") == ops("k_j_decaps") + ops("k_decrypt_core") + xof
    # {fix-up, PRFs} runs in both operations: the PRFs count twice, the fix-up not at all
    assert ops("k_xof_fix+k_prf") == ops("k_prf")
    # a whole encaps+decaps step: every SampleNTT and PRF pass once per operation
    step = (ops("k_front_encaps+k_xof") + ops("k_j_decaps+k_decrypt_core+k_xof") + ops("k_xof_fix+k_prf")
            + ops("k_g_decaps") + ops("k_encrypt_core"))
    alone = (ops("k_front_encaps") + ops("k_j_decaps") + ops("k_decrypt_core") + ops("k_xof") + ops("k_prf")
             + ops("k_g_decaps") + ops("k_encrypt_core"))
    assert step == alone
    # decaps-only mode: the Decaps launch is unchanged, the shared kernels count once
    assert ops("k_xof_fix+k_prf", "decaps-tampered") == ops("k_prf") // 2


def test_survey_w_pricing_of_the_cores():
    k = 3
    ntt, bm = 896 * 8, 3584
    assert bench.survey_core_ops("ML-KEM-768", "k_encrypt_core", "encdec") == 2 * (7 * ntt + 12 * bm)
    assert bench.survey_core_ops("ML-KEM-768", "k_decrypt_core", "encdec") == (k + 1) * ntt + k * bm
    assert bench.survey_core_ops("ML-KEM-768", "k_xof", "encdec") is None
    kernels, roof, _ = bench.kernel_report("ML-KEM-768", "encdec", {"k_encrypt_core": (3.8, 2)}, 1 << 20)
    e = kernels["k_encrypt_core"]
    assert e["survey_w_frac"] == pytest.approx(e["frac"] * (2 * (7 * ntt + 12 * bm)) / bench.kernel_ops_per_hs(
        "ML-KEM-768", "k_encrypt_core", "encdec")[0])


def test_hqc_products_priced_against_lds():
    """HQC's sparse-dense products are bound by their LDS window reads (>= 1 dword per output word and
    position: 2 LDS clocks per wave-position against 1.5 CU clocks of VALU), so bench.py prices them
    against LDS_LOOKUP_PEAK and reports the VALU fraction beside it."""
    ops, bound = bench.kernel_ops_per_hs("HQC-128", "k_hqc_enc_mul", "encdec")
    assert bound == "lds" and ops == 2 * (2 * 75 * ((17669 + 31) // 32))  # Encaps + re-encryption
    kernels, roof, _ = bench.kernel_report("HQC-128", "encdec", {"k_hqc_enc_mul": (0.8, 2)}, 1 << 16)
    k = kernels["k_hqc_enc_mul"]
    assert k["frac"] == pytest.approx(ops * (1 << 16) / 0.8e-3 / bench.LDS_LOOKUP_PEAK)
    assert k["valu_frac"] == pytest.approx(k["frac"] * 2 * bench.LDS_LOOKUP_PEAK / bench.VALU_PEAK)
    assert roof["bound"] == "lds" and roof["valu_frac"] == pytest.approx(k["valu_frac"])
