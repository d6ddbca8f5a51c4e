"""configurator.py semantics and config presets."""

import os

import pytest

from nanosandbox_amd.config import TRAIN_DEFAULTS, apply_overrides, config_keys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def ns():
    return dict(TRAIN_DEFAULTS)


def test_literal_eval_and_types():
    c = apply_overrides(ns(), ["--batch_size=32", "--dropout=0.1", "--compile=False", "--device=cpu"], verbose=False)
    assert c["batch_size"] == 32 and isinstance(c["batch_size"], int)
    assert c["dropout"] == 0.1
    assert c["compile"] is False
    assert c["device"] == "cpu"  # not literal-evaluable -> stays a string


def test_type_mismatch_rejected():
    # nanoGPT asserts exact type equality: 0 is an int, dropout is a float
    with pytest.raises(AssertionError):
        apply_overrides(ns(), ["--dropout=0"], verbose=False)
    with pytest.raises(AssertionError):
        apply_overrides(ns(), ["--batch_size=1.5"], verbose=False)


def test_unknown_key():
    with pytest.raises(ValueError, match="Unknown config key: nope"):
        apply_overrides(ns(), ["--nope=1"], verbose=False)


def test_override_must_have_dashes():
    with pytest.raises(AssertionError):
        apply_overrides(ns(), ["batch_size=3"], verbose=False)


def test_config_file_then_override(tmp_path):
    f = tmp_path / "cfg.py"
    f.write_text("n_layer = 3\nbatch_size = 7\nimport math\nlearning_rate = math.sqrt(4) * 1e-4\n")
    c = apply_overrides(ns(), [str(f), "--batch_size=9"], verbose=False)
    assert c["n_layer"] == 3 and c["batch_size"] == 9
    assert abs(c["learning_rate"] - 2e-4) < 1e-12
    assert "math" not in c  # modules are not config


def test_config_file_with_dashes_rejected():
    with pytest.raises(AssertionError):
        apply_overrides(ns(), ["--config/x.py"], verbose=False)


def test_new_keys_are_typed():
    c = apply_overrides(ns(), ["--ddp_bucket_mb=128", "--data_dir=/data/datasets", "--grad_ckpt=True",
                               "--ddp_impl=torch"], verbose=False)
    assert c["ddp_bucket_mb"] == 128 and c["data_dir"] == "/data/datasets"
    assert c["grad_ckpt"] is True and c["ddp_impl"] == "torch"


@pytest.mark.parametrize("name", sorted(os.listdir(os.path.join(ROOT, "config"))))
def test_presets_parse(name):
    c = apply_overrides(ns(), [os.path.join(ROOT, "config", name)], verbose=False)
    assert set(config_keys(c)) >= set(TRAIN_DEFAULTS)


def test_shakespeare_char_preset_values():
    c = apply_overrides(ns(), [os.path.join(ROOT, "config", "train_shakespeare_char.py")], verbose=False)
    assert (c["n_layer"], c["n_head"], c["n_embd"], c["block_size"], c["batch_size"]) == (6, 6, 384, 256, 64)
    assert c["dropout"] == 0.2 and c["beta2"] == 0.99 and c["always_save_checkpoint"] is False


def test_gpt2_preset_tokens_per_iter():
    c = apply_overrides(ns(), [os.path.join(ROOT, "config", "train_gpt2.py")], verbose=False)
    assert c["batch_size"] * c["block_size"] * c["gradient_accumulation_steps"] == 491520


def test_root_configurator_exec(tmp_path, monkeypatch):
    # scripts that `exec(open('configurator.py').read())` keep working
    g = {"batch_size": 1, "dropout": 0.0, "__name__": "__main__"}
    monkeypatch.setattr("sys.argv", ["train.py", "--batch_size=4"])
    exec(open(os.path.join(ROOT, "configurator.py")).read(), g)
    assert g["batch_size"] == 4
