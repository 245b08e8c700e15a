"""The launchers (run-cpu.sh / run-rocm.sh / run-remote.sh) load .env files with
scripts/load_env.sh under `set -euo pipefail`: every shipped template must load
without a shell error, values with spaces must come through whole, and variables
already in the environment must win over the file."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
TEMPLATES = [".env.example", ".env.remote.example"]


def _load(path, extra_env=None, probe="SYSTEM_PROMPT"):
    script = (f'set -euo pipefail; source "{ROOT}/scripts/load_env.sh"; '
              f'load_env_file "{path}"; printf "%s" "${{{probe}:-}}"')
    env = {"PATH": os.environ.get("PATH", "/usr/bin:/bin")}
    env.update(extra_env or {})
    return subprocess.run(["bash", "-c", script], capture_output=True, text=True, env=env,
                          timeout=30)


@pytest.mark.parametrize("name", TEMPLATES)
def test_template_loads_under_set_e(name):
    r = _load(os.path.join(ROOT, name))
    assert r.returncode == 0, r.stderr
    assert r.stdout.startswith("You are a helpful voice assistant."), r.stdout


@pytest.mark.parametrize("name", TEMPLATES)
def test_template_is_also_plain_bash_sourceable(name):
    # docker/compose users and old scripts `source` the file directly: keep it valid bash
    script = f'set -euo pipefail; set -a; source "{os.path.join(ROOT, name)}"; set +a; printf "%s" "$SYSTEM_PROMPT"'
    r = subprocess.run(["bash", "-c", script], capture_output=True, text=True, timeout=30,
                       env={"PATH": os.environ.get("PATH", "/usr/bin:/bin")})
    assert r.returncode == 0, r.stderr
    assert "Keep responses concise" in r.stdout


def test_environment_wins_and_values_are_literal(tmp_path):
    f = tmp_path / "e.env"
    f.write_text("# comment\nA=from file\nB='single $HOME quoted'\nexport C=\"x y\"\nbad line\n"
                 "D=$(echo pwned)\n")
    assert _load(str(f), {"A": "from env"}, "A").stdout == "from env"
    assert _load(str(f), probe="B").stdout == "single $HOME quoted"
    assert _load(str(f), probe="C").stdout == "x y"
    assert _load(str(f), probe="D").stdout == "$(echo pwned)"
