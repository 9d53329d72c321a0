"""bench.py's PMC lookups pick the kernel instance each roofline prices (CPU only).

A roofline's `traffic` must reproduce from profiles/pmc_summary.json: the lookup
matches the bare kernel name and its template arguments exactly, so the left
pyramid chain (Scharr on) is never confused with the right pyramid's instances
of the same templates, nor the temporal 21x21 LK with the stereo 11x11 one.
"""
import json

import pytest

import bench

KERNELS = {
    # the right pyramid (no Scharr) listed first, as rocprofv3's summary sorts it
    "void svo::pyr_scharr_kernel<true, false, true>": {"hbm_bytes_per_launch": 127_298_869},
    "void svo::pyr_scharr_kernel<true, true, true>": {"hbm_bytes_per_launch": 428_894_941},
    "void svo::pyr_chain_kernel<3, false, 2>": {"hbm_bytes_per_launch": 33_192_514},
    "void svo::pyr_chain_kernel<3, true, 2>": {"hbm_bytes_per_launch": 72_826_649},
    "void svo::lk_multi_kernel<4, 1, 4, 1, 11, 11, 11>": {"hbm_bytes_per_launch": 137_986_670},
    "void svo::lk_multi_kernel<4, 1, 3, 2, 21, 21, 7>": {"hbm_bytes_per_launch": 814_485_556},
    "void svo::fast_detect_q_kernel<32, true>": {"hbm_bytes_per_launch": 168_013_144},
    "svo::post_lk_kernel": {"hbm_bytes_per_launch": 39_663_716},
}


def test_kernel_key_parses_template_arguments():
    assert bench.kernel_key("void svo::pyr_chain_kernel<3, true, 2>") == ("pyr_chain_kernel", ("3", "true", "2"))
    assert bench.kernel_key("svo::post_lk_kernel") == ("post_lk_kernel", ())
    assert bench.kernel_key("void svo::append_kernel<256>") == ("append_kernel", ("256",))


def test_pmc_select_exact_instances():
    k, _ = bench.pmc_select(KERNELS, "pyr_scharr_kernel", bench.PYR_LEFT_TARGS)
    assert k == "void svo::pyr_scharr_kernel<true, true, true>"
    k, _ = bench.pmc_select(KERNELS, "pyr_chain_kernel", bench.CHAIN_LEFT_TARGS)
    assert k == "void svo::pyr_chain_kernel<3, true, 2>"
    k, _ = bench.pmc_select(KERNELS, "lk_multi_kernel", bench.LK_TEMPORAL_TARGS)
    assert k == "void svo::lk_multi_kernel<4, 1, 3, 2, 21, 21, 7>"
    k, _ = bench.pmc_select(KERNELS, "post_lk_kernel")
    assert k == "svo::post_lk_kernel"
    assert bench.pmc_select(KERNELS, "lk_fast_kernel", ("21", "21", None)) == (None, None)
    # round 6's keys: the LOOP argument appended, the temporal LK built for 4 waves per SIMD
    k6 = {"void svo::lk_multi_kernel<4, 1, 6, 1, 11, 11, 11, true>": {"hbm_bytes_per_launch": 1},
          "void svo::lk_multi_kernel<4, 1, 4, 2, 21, 21, 7, false>": {"hbm_bytes_per_launch": 2}}
    assert bench.pmc_select(k6, "lk_multi_kernel", bench.LK_TEMPORAL_TARGS)[1] == {"hbm_bytes_per_launch": 2}
    # a bare name with two instances and no constraint is refused, not guessed
    with pytest.raises(ValueError):
        bench.pmc_select(KERNELS, "pyr_scharr_kernel")


def test_pmc_traffic_left_chain_and_scaling(tmp_path, monkeypatch):
    prof = tmp_path / "profiles"
    prof.mkdir()
    summ = {"configs": {"kitti": {"source": "x: rocprofv3 --pmc ... 'python bench.py --config kitti --seq 256'",
                                  "kernels": KERNELS}}}
    (prof / "pmc_summary.json").write_text(json.dumps(summ))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    ps = bench.pmc_traffic("kitti", "pyr_scharr_kernel", 256, bench.PYR_LEFT_TARGS)
    ch = bench.pmc_traffic("kitti", "pyr_chain_kernel", 256, bench.CHAIN_LEFT_TARGS)
    # the fused chain at maxLevel 3: (c - 1) = 2 pyr_scharr launches + the chain kernel
    assert 2 * ps + ch == 2 * 428_894_941 + 72_826_649  # 930.6 MB, not the right pyramid's 327.4 MB
    assert bench.pmc_traffic("kitti", "lk_multi_kernel", 256, bench.LK_TEMPORAL_TARGS) == 814_485_556
    assert bench.pmc_traffic("kitti", "lk_multi_kernel", 128, bench.LK_TEMPORAL_TARGS) == 814_485_556 // 2
    assert bench.pmc_traffic("1080p", "lk_multi_kernel", 64, bench.LK_TEMPORAL_TARGS) is None


def test_committed_summary_resolves_every_priced_instance():
    """Every config in the committed summary resolves each priced instance to one key."""
    with open(bench.os.path.join(bench.ROOT, "profiles", "pmc_summary.json")) as f:
        d = json.load(f)
    for cfg, c in d["configs"].items():
        ks = c["kernels"]
        assert bench.pmc_select(ks, "lk_multi_kernel", bench.LK_TEMPORAL_TARGS)[0] is not None, cfg
        assert bench.pmc_select(ks, "pyr_scharr_kernel", bench.PYR_LEFT_TARGS)[0] is not None, cfg
        assert bench.pmc_select(ks, "pyr_chain_kernel", bench.CHAIN_LEFT_TARGS)[0] is not None, cfg
        assert bench.pmc_select(ks, "fast_detect_q_kernel")[0] is not None, cfg


def test_valu_lookup_temporal_lk(tmp_path, monkeypatch):
    # the SQ mix pass keys kernels with all their template arguments (round 6: LOOP appended)
    prof = tmp_path / "profiles"
    prof.mkdir()
    summ = {"source": "SQ_INSTS_VALU / SQ_WAVES of: python bench.py --seq 256 --steps 8",
            "kernels": {"lk_multi_kernel<4, 1, 6, 1, 11, 11, 11, true>": {"valu_per_dispatch": 1},
                        "lk_multi_kernel<4, 1, 3, 2, 21, 21, 7, false>": {"valu_per_dispatch": 2}}}
    (prof / "valu_summary.json").write_text(json.dumps(summ))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    r = bench.roofline_valu("lk_multi_kernel<4, 1", 128, 1e-3)
    assert r is not None and r["valu_per_launch"] == 1  # 2 per 256 sequences, scaled to 128
