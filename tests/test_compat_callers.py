"""The callers' own import blocks, executed unchanged after ``compat.install()`` (CPU).

SURVEY.md 8(b): the build drops into ``prediction.ipynb`` and ``scripts/04_train.py`` with no
edit.  Those callers import helpers the build does not provide (``log`` / ``synth_one_sample``
from ``scripts/utils/tools.py:140,180``, ``plot_mel`` from ``:541``): they must resolve to the
caller's own definitions, while the hot-path names resolve to this package.  A fake caller tree
in ``tmp_path`` stands in for the reference checkout (the real one needs matplotlib / cv2 /
torchvision at import, which this image lacks)."""

import sys
import textwrap

import pytest

_ROOTS = ("model", "transformer", "hifigan", "utils", "scripts", "audio", "dataset", "evaluate")

# scripts/04_train.py:11-16 (verbatim)
TRAIN_IMPORTS = """\
from utils.model import get_model, get_vocoder, get_param_num
from utils.tools import to_device, log, synth_one_sample
from model import FastSpeech2Loss
from dataset import Dataset
from scipy.io.wavfile import write
from evaluate import evaluate
"""

# scripts/evaluate.py:9-12 (verbatim)
EVALUATE_IMPORTS = """\
from utils.model import get_model, get_vocoder
from utils.tools import to_device, log, synth_one_sample
from model import FastSpeech2Loss
from dataset import Dataset
"""

# prediction.ipynb source lines 47, 65, 215, 307 (verbatim, de-indented)
NOTEBOOK_IMPORTS = """\
from scripts.utils.model import get_model, get_vocoder
from scripts.dataset import Dataset
from scripts.utils.tools import to_device, plot_mel, expand
from scripts.utils.model import vocoder_infer
"""

_CALLER_TOOLS = '''\
"""stand-in for the reference's scripts/utils/tools.py (non-path helpers only)"""
import numpy as np
import audio as Audio                                   # tools.py:12 (aliased)

CALLS = []


def log(logger, step=None, losses=None, fig=None, audio=None, sampling_rate=22050, tag=""):
    CALLS.append(("log", step))


def synth_one_sample(targets, predictions, vocoder, model_config, preprocess_config):
    from .model import vocoder_infer                    # tools.py:224: lands on the build
    CALLS.append(("synth", vocoder_infer.__module__))
    return None, None, None, None


def plot_mel(data, stats, titles):
    CALLS.append(("plot_mel", len(data)))
    return "fig"


def to_device(data, device):                            # shadowed by the build's to_device
    raise AssertionError("caller's to_device must not be used")
'''

_CALLER_EVALUATE = EVALUATE_IMPORTS + '''

def evaluate(model, step, configs, logger=None, vocoder=None, device=None):
    log(logger, step)
    return "evaluated"
'''


@pytest.fixture
def caller_tree(tmp_path, monkeypatch):
    scripts = tmp_path / "scripts"
    (scripts / "utils").mkdir(parents=True)
    (scripts / "utils" / "tools.py").write_text(_CALLER_TOOLS)
    (scripts / "evaluate.py").write_text(_CALLER_EVALUATE)
    saved = {k: sys.modules.get(k) for k in list(sys.modules) if k.split(".")[0] in _ROOTS}
    monkeypatch.chdir(tmp_path)                       # the reference runs from its repo root
    monkeypatch.syspath_prepend(str(scripts))         # 04_train.py's own directory
    from visual_onoma_to_wave_amd import compat
    compat.install()
    try:
        yield tmp_path
    finally:
        compat._caller_mods.clear()
        compat._caller_errors.clear()
        for k in list(sys.modules):
            if k.split(".")[0] in _ROOTS:
                del sys.modules[k]
        sys.modules.update({k: v for k, v in saved.items() if v is not None})


def _exec(src):
    ns = {}
    exec(compile(src, "<caller>", "exec"), ns)
    return ns


def test_train_script_imports_resolve(caller_tree):
    ns = _exec(TRAIN_IMPORTS)
    for name in ("get_model", "get_vocoder", "get_param_num", "to_device", "FastSpeech2Loss",
                 "Dataset"):
        assert ns[name].__module__.startswith("visual_onoma_to_wave_amd"), name
    assert ns["log"].__module__ == "utils._caller_tools"
    assert ns["synth_one_sample"].__module__ == "utils._caller_tools"
    assert ns["evaluate"](None, 7, None) == "evaluated"
    caller = sys.modules["utils._caller_tools"]
    assert ("log", 7) in caller.CALLS
    ns["synth_one_sample"](None, None, None, None, None)
    assert ("synth", "visual_onoma_to_wave_amd.utils.model") in caller.CALLS


def test_notebook_imports_resolve(caller_tree):
    ns = _exec(NOTEBOOK_IMPORTS)
    for name in ("get_model", "get_vocoder", "vocoder_infer", "Dataset", "to_device", "expand"):
        assert ns[name].__module__.startswith("visual_onoma_to_wave_amd"), name
    assert ns["plot_mel"]([1, 2], None, None) == "fig"
    assert ns["plot_mel"].__module__ == "scripts.utils._caller_tools" or \
        ns["plot_mel"].__module__ == "utils._caller_tools"


def test_missing_name_without_caller_tree(tmp_path, monkeypatch):
    saved = {k: sys.modules.get(k) for k in list(sys.modules) if k.split(".")[0] in _ROOTS}
    monkeypatch.chdir(tmp_path)
    from visual_onoma_to_wave_amd import compat
    compat.install()
    try:
        with pytest.raises(ImportError, match="plot_mel"):
            _exec("from utils.tools import plot_mel\n")
        with pytest.raises(AttributeError, match="not on the synthesis path"):
            getattr(sys.modules["utils.tools"], "plot_mel")
        ns = _exec("from utils.tools import to_device, expand, pad, get_mask_from_lengths\n")
        assert all(f.__module__ == "visual_onoma_to_wave_amd.utils.tools" for f in ns.values()
                   if callable(f))
    finally:
        compat._caller_mods.clear()
        compat._caller_errors.clear()
        for k in list(sys.modules):
            if k.split(".")[0] in _ROOTS:
                del sys.modules[k]
        sys.modules.update({k: v for k, v in saved.items() if v is not None})


def test_caller_root_argument(tmp_path, monkeypatch):
    """``install(caller_root=...)`` finds the tree when the cwd is elsewhere."""
    (tmp_path / "ref" / "scripts" / "utils").mkdir(parents=True)
    (tmp_path / "ref" / "scripts" / "utils" / "tools.py").write_text(textwrap.dedent("""
        def plot_mel(data, stats, titles):
            return "ok"
    """))
    (tmp_path / "elsewhere").mkdir()
    monkeypatch.chdir(tmp_path / "elsewhere")
    saved = {k: sys.modules.get(k) for k in list(sys.modules) if k.split(".")[0] in _ROOTS}
    from visual_onoma_to_wave_amd import compat
    compat.install(caller_root=tmp_path / "ref")
    try:
        assert _exec("from scripts.utils.tools import plot_mel\n")["plot_mel"](0, 0, 0) == "ok"
    finally:
        compat._caller_root = None
        compat._caller_mods.clear()
        compat._caller_errors.clear()
        for k in list(sys.modules):
            if k.split(".")[0] in _ROOTS:
                del sys.modules[k]
        sys.modules.update({k: v for k, v in saved.items() if v is not None})


def test_failing_caller_tree_probes_stay_probes(tmp_path, monkeypatch):
    """A caller tools.py whose own imports fail (matplotlib / tensorboard absent) makes ``hasattr`` /
    ``getattr(..., default)`` return False / the default -- AttributeError chained from the real
    error -- and is executed once, not on every probe; a name that is not one of the reference's
    off-path helpers never executes the caller's file."""
    (tmp_path / "scripts" / "utils").mkdir(parents=True)
    counter = tmp_path / "count.txt"
    (tmp_path / "scripts" / "utils" / "tools.py").write_text(textwrap.dedent(f"""
        open({str(counter)!r}, "a").write("x")
        import a_module_that_is_not_installed  # noqa
        def plot_mel(data, stats, titles):
            return "ok"
    """))
    monkeypatch.chdir(tmp_path)
    saved = {k: sys.modules.get(k) for k in list(sys.modules) if k.split(".")[0] in _ROOTS}
    from visual_onoma_to_wave_amd import compat
    compat.install()
    try:
        tools = sys.modules["utils.tools"]
        assert not hasattr(tools, "plot_mel")
        assert getattr(tools, "synth_one_sample", "default") == "default"
        with pytest.raises(AttributeError) as ei:
            tools.plot_mel
        assert isinstance(ei.value.__cause__, ImportError)
        assert counter.read_text() == "x"  # executed once
        assert not hasattr(tools, "no_such_helper")
        assert counter.read_text() == "x"
    finally:
        compat._caller_mods.clear()
        compat._caller_errors.clear()
        for k in list(sys.modules):
            if k.split(".")[0] in _ROOTS:
                del sys.modules[k]
        sys.modules.update({k: v for k, v in saved.items() if v is not None})
