"""Drop-in CLI contract (no GPU needed): `make train-best / evaluate / tune` pass the reference's flags, so every
flag and default the reference's argparse declares must parse here with the same value. The expected tables restate
the reference's parsers (src/ml/train.py:347-361, src/ml/evaluate.py:345-355, src/ml/tune.py:327-337) and its
default grid (src/ml/tune.py:33-39)."""
import argparse
import os
import sys

import pytest

ANY = object()  # path defaults (src/config.py directories): the flag must exist, its value is site-specific
TRAIN_FLAGS = {  # src/ml/train.py:347-361, with src/config.py:29-33's defaults (env unset)
    "--data": ANY, "--embeddings": ANY, "--output": ANY, "--latent-dim": 50, "--hidden-dims": [256],
    "--batch-size": 64, "--epochs": 10, "--learning-rate": 1e-3, "--weight-decay": 0.0, "--beta": 0.2,
    "--dropout": 0.5, "--use-annealing": False, "--patience": 20, "--device": None, "--ignore-embeddings": False,
}
EVAL_FLAGS = {  # src/ml/evaluate.py:345-355
    "--model": ANY, "--data": ANY, "--embeddings": ANY, "--k-values": [5, 10, 20], "--device": None,
    "--output": None, "--n-negatives": 99,
}
TUNE_FLAGS = {  # src/ml/tune.py:327-337
    "--data": ANY, "--embeddings": ANY, "--output": ANY, "--epochs": 10, "--patience": 3, "--batch-size": 512,
    "--device": None, "--latent-dims": [32, 64, 128], "--dropouts": [0.3, 0.5], "--betas": [0.1, 0.2, 0.3],
    "--learning-rates": [1e-3, 5e-4],
}


def _capture_parser(monkeypatch, module):
    """Run module.main() up to parse_args and return the parser it built (main stops there)."""
    seen = {}

    class _Stop(Exception):
        pass

    def fake_parse(self, args=None, namespace=None):
        seen["parser"] = self
        raise _Stop

    monkeypatch.setattr(argparse.ArgumentParser, "parse_args", fake_parse)
    monkeypatch.setattr(sys, "argv", ["prog"])
    with pytest.raises(_Stop):
        module.main()
    return seen["parser"]


@pytest.mark.parametrize("modname,flags", [("src.ml.train", TRAIN_FLAGS), ("src.ml.evaluate", EVAL_FLAGS),
                                           ("src.ml.tune", TUNE_FLAGS)])
def test_cli_accepts_reference_flags(monkeypatch, modname, flags):
    if any(os.environ.get(v) for v in ("BATCH_SIZE", "LEARNING_RATE", "EPOCHS", "LATENT_DIM", "HIDDEN_DIM")):
        pytest.skip("src/config.py defaults overridden from the environment")
    import importlib
    mod = importlib.import_module(modname)
    parser = _capture_parser(monkeypatch, mod)
    by_flag = {o: a for a in parser._actions for o in a.option_strings}
    for flag, default in flags.items():
        assert flag in by_flag, f"{modname}: reference flag {flag} missing"
        if default is not ANY:
            assert by_flag[flag].default == default, f"{modname} {flag}: {by_flag[flag].default} != {default}"
    dev = by_flag["--device"]
    assert set(dev.choices) == {"cuda", "cpu", "mps"}, f"{modname}: --device choices {dev.choices}"


def test_default_search_space_is_the_reference_grid():
    from src.ml.tune import DEFAULT_SEARCH_SPACE
    assert DEFAULT_SEARCH_SPACE == {  # src/ml/tune.py:33-39
        "latent_dim": [32, 64, 128],
        "hidden_dims": [[256], [512], [256, 128]],
        "dropout": [0.3, 0.5],
        "beta": [0.1, 0.2, 0.3],
        "learning_rate": [1e-3, 5e-4],
    }
    assert list(DEFAULT_SEARCH_SPACE) == ["latent_dim", "hidden_dims", "dropout", "beta", "learning_rate"]


@pytest.mark.parametrize("modname", ["src.ml.train", "src.ml.evaluate", "src.ml.tune"])
@pytest.mark.parametrize("device", ["cpu", "mps"])
def test_non_hip_device_fails_loudly(modname, device):
    import importlib
    mod = importlib.import_module(modname)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        mod._get_device(device)


@pytest.mark.parametrize("conc", [0, 9])
def test_tune_concurrency_bounds(tmp_path, conc):
    """--concurrent packs 1..8 configuration processes onto one GPU; anything else fails before data loads."""
    from src.ml.tune import run_grid_search
    with pytest.raises(ValueError, match="concurrent"):
        run_grid_search(str(tmp_path / "no_data"), str(tmp_path / "no_emb.npy"), str(tmp_path / "out"),
                        concurrent=conc)


def test_tune_cli_concurrency_flags():
    """The MI355X additions to the reference's tune flags: --concurrent (default 1, the serial search) and --seed."""
    import sys
    from unittest import mock
    import src.ml.tune as t
    with mock.patch.object(t, "run_grid_search") as run, \
            mock.patch.object(sys, "argv", ["tune", "--concurrent", "4", "--seed", "3"]):
        t.main()
    kw = run.call_args.kwargs
    assert kw["concurrent"] == 4 and kw["seed"] == 3
    with mock.patch.object(t, "run_grid_search") as run, mock.patch.object(sys, "argv", ["tune"]):
        t.main()
    assert run.call_args.kwargs["concurrent"] == 1 and run.call_args.kwargs["seed"] is None
