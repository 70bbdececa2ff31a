"""Every runtime knob the C ABI reads from the environment is documented in README.md.

The option names come from `kOptionNames` in frei_runtime.hip (each read as FREI_<NAME> when a
context is created) plus the names the sources read with getenv / os.environ directly."""
import pathlib
import re

ROOT = pathlib.Path(__file__).resolve().parents[1]


def _option_names():
    src = (ROOT / "frei_amd/csrc/frei_runtime.hip").read_text()
    m = re.search(r"kOptionNames\[\]\s*=\s*\{(.*?)nullptr\}", src, re.S)
    assert m, "kOptionNames not found"
    names = {"FREI_" + n.upper() for n in re.findall(r'"([a-z0-9_]+)"', m.group(1))}
    assert len(names) >= 10
    return names


def _direct_env_names():
    names = set()
    for f in list((ROOT / "frei_amd").rglob("*.py")) + list((ROOT / "frei_amd/csrc").glob("*.hip")):
        names |= set(re.findall(r'"(FREI_[A-Z0-9_]+)"', f.read_text()))
    return names


def test_every_environment_knob_is_documented():
    readme = (ROOT / "README.md").read_text()
    missing = sorted(n for n in _option_names() | _direct_env_names() if f"`{n}`" not in readme)
    assert not missing, f"README.md does not document {missing}"
