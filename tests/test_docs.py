"""Documentation stays correct: every runnable Python block of the tutorials executes (CPU, in order,
one interpreter per page -- the Molecule registry is process-wide), and the generated API
reference matches the docstrings (``docs/gen_api.py --check``)."""
import os
import re
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_BLOCK = re.compile(r"(<!-- norun -->\s*\n)?```python\n(.*?)```", re.S)


def _blocks(path: str) -> list[str]:
    text = open(path, encoding="utf-8").read()
    return [m.group(2) for m in _BLOCK.finditer(text) if not m.group(1)]


@pytest.mark.parametrize("page", ["tutorials.md", "multi_gpu.md", "index.md"])
def test_doc_code_blocks_run(page, tmp_path):
    path = os.path.join(ROOT, "docs", page)
    blocks = _blocks(path)
    if not blocks:
        pytest.skip("no runnable blocks")
    script = tmp_path / "doc.py"
    script.write_text("\n\n".join(f"# --- block {i}\n{b}" for i, b in enumerate(blocks)))
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="4")
    p = subprocess.run([sys.executable, str(script)], capture_output=True, text=True, env=env, cwd=str(tmp_path),
                       timeout=900)
    assert p.returncode == 0, f"{page}:\n{p.stdout[-2000:]}\n{p.stderr[-4000:]}"


def test_api_reference_is_current():
    p = subprocess.run([sys.executable, os.path.join(ROOT, "docs", "gen_api.py"), "--check"], capture_output=True,
                       text=True, cwd=ROOT)
    assert p.returncode == 0, p.stderr
