"""bench.py's algorithmic-byte models against SURVEY.md 8(d)'s per-config figures."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def test_state_resident_model_123bus():
    assert bench.bytes_alg_per_scenario(122, 123) == 11788          # config 2 / 4


def test_streaming_model_2048bus():
    # 196,588 + 393,024 k_s B per scenario (config 3)
    nb, nn = 2047, 2048
    assert bench.bytes_alg_per_scenario(nb, nn) == 196588
    assert bench.bytes_alg_streaming(nb, nn, k_sum=5.0, n_scen=1) == 196588 + 393024 * 5
    assert bench.bytes_alg_streaming(nb, nn, k_sum=5.0 * 8, n_scen=8) == 8 * (196588 + 393024 * 5)


def test_configs():
    assert bench.CONFIGS[2][:3] == (123, 123, 4096)
    assert bench.CONFIGS[3][:3] == (2048, 2048, 65536)
    assert bench.CONFIGS[4][2] * 8 == 1 << 20                         # 2^20 scenarios over 8 GPUs


def test_instruction_efficiency_lookup(tmp_path, monkeypatch):
    """roofline.fp64.instruction_efficiency: useful flops / (128 x the committed
    SQ_INSTS_VALU per launch); absent when no SQ pass was committed."""
    import json
    import bench
    d = {"by_workload": {"123-bus x 4096": {"kernel": "dpf_wave_kernel", "valu_insts_per_launch": 1.0e6,
                                            "valu_tag": "t"}}}
    (tmp_path / "profiles").mkdir()
    (tmp_path / "profiles" / "pmc_traffic.json").write_text(json.dumps(d))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    e = bench._instruction_efficiency("123-bus x 4096", "dpf_wave_kernel", 64.0e6)
    assert e["instruction_efficiency"] == 0.5 and e["valu_source"] == "t"
    assert bench._instruction_efficiency("123-bus x 4096", "dpf_wblk_kernel", 1.0) == {}
    assert bench._instruction_efficiency("2048-bus x 1", "dpf_wave_kernel", 1.0) == {}
