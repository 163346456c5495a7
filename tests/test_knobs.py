"""Every DV_* environment variable the package reads is registered in deconv_api_amd/knobs.py, the
A/B switches are read only through the ablation gate, and at most 30 production switches remain
(85 names, 45 getenv sites in csrc, 35 environ reads outside config.py)."""
import pathlib
import re

from deconv_api_amd import knobs

PKG = pathlib.Path(__file__).resolve().parents[1] / "deconv_api_amd"
GATED = [r'dv_ab_env\("(DV_[A-Z0-9_]+)"\)', r'knobs\.ablation\("(DV_[A-Z0-9_]+)"']
PLAIN = [r'std::getenv\("(DV_[A-Z0-9_]+)"\)', r'os\.environ\.get\("(DV_[A-Z0-9_]+)"', r'os\.environ\["(DV_[A-Z0-9_]+)"\]']


def _reads():
    gated, plain, mentioned = set(), set(), set()
    for p in PKG.rglob("*"):
        if p.suffix not in (".py", ".hip", ".h", ".cpp") or p.name == "knobs.py" or "__pycache__" in p.parts:
            continue
        s = p.read_text()
        for pat in GATED:
            gated.update(re.findall(pat, s))
        for pat in PLAIN:
            plain.update(re.findall(pat, s))
        mentioned.update(re.findall(r"DV_[A-Z0-9_]+", s))
    return gated, plain, mentioned


def test_every_env_read_is_registered_and_gated():
    gated, plain, _ = _reads()
    assert gated <= set(knobs.ABLATION), sorted(gated - set(knobs.ABLATION))
    assert not (plain & set(knobs.ABLATION)), f"A/B switches read without the gate: {sorted(plain & set(knobs.ABLATION))}"
    allowed = set(knobs.RUNTIME) | set(knobs.BUILD) | knobs.config_names()
    assert plain <= allowed, f"unregistered DV_* reads: {sorted(plain - allowed)}"


def test_no_stale_registry_entries():
    _, _, mentioned = _reads()
    registered = set(knobs.RUNTIME) | set(knobs.ABLATION) | set(knobs.BUILD)
    assert registered <= mentioned, f"registered but never read: {sorted(registered - mentioned)}"


def test_runtime_switch_budget():
    assert len(knobs.RUNTIME) <= 30, len(knobs.RUNTIME)
    assert not (set(knobs.RUNTIME) & knobs.config_names())


def test_ablation_gate(monkeypatch):
    monkeypatch.setenv("DV_RELU_BITS", "0")
    monkeypatch.setenv("DV_ABLATIONS", "0")
    assert knobs.ablation("DV_RELU_BITS", "1") == "1"
    monkeypatch.setenv("DV_ABLATIONS", "1")
    assert knobs.ablation("DV_RELU_BITS", "1") == "0"
