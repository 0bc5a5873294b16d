"""Example chemistries and the README walkthrough (BASELINE plumbing config) on the CPU."""
import subprocess
import sys

import pytest
import torch

import magicsoup_amd as ms


_README_CHECK = """
import torch
from magicsoup_amd.examples import readme

w = readme.make_world("cpu", n_cells=100, map_size=128)
assert w.n_cells == 100
total0 = w.molecule_map.double().sum() + w.cell_molecules.double().sum()
readme.run(w, 15)
assert w.n_cells > 0
assert int(w.cell_map.sum()) == w.n_cells
assert torch.isfinite(w.molecule_map).all() and (w.molecule_map >= 0).all()
# the reaction only converts molecules; diffusion/permeation conserve them, kills spill them
# (no degradation call in this loop): the total amount changes only through the reaction
total = w.molecule_map.double().sum() + w.cell_molecules.double().sum()
assert abs(float(total - total0)) / float(total0) < 0.05
print("ok")
"""


def test_readme_walkthrough_runs_on_cpu():
    # own process: the README molecules (e.g. NADP at 100 kJ) clash with the example chemistries'
    # definitions of the same names in the process-wide Molecule registry
    out = subprocess.run([sys.executable, "-c", _README_CHECK], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    assert out.stdout.strip() == "ok"


@pytest.mark.parametrize("name, n_mol, n_react", [("wood_ljungdahl", 14, 6), ("reverse_krebs", 15, 8),
                                                   ("n2_fixing", 10, 2)])
def test_example_chemistries_in_subprocess(name, n_mol, n_react):
    # separate processes: the example chemistries reuse molecule names with different energies,
    # which the Molecule registry rejects within one process (as in the reference)
    code = (f"from magicsoup_amd.examples.{name} import CHEMISTRY as C; "
            "print(len(C.molecules), len(C.reactions))")
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert out.stdout.split() == [str(n_mol), str(n_react)]


def test_co2_fixing_chemistry_in_subprocess():
    code = ("from magicsoup_amd.examples.co2_fixing import CHEMISTRY as C; "
            "import magicsoup_amd as ms; w = ms.World(chemistry=C, map_size=16); "
            "w.spawn_cells([ms.random_genome(800) for _ in range(30)]); w.enzymatic_activity(); "
            "w.diffuse_molecules(); print(len(C.molecules), len(C.reactions), w.n_cells)")
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    assert out.stdout.split() == ["41", "46", "30"]


def test_synthetic_wide_chemistry():
    from magicsoup_amd.examples.synthetic import make_chemistry

    chem = make_chemistry(n_molecules=64, n_reactions=256, seed=3)
    assert len(chem.molecules) == 64 and len(chem.reactions) == 256
    w = ms.World(chemistry=chem, map_size=16)
    w.spawn_cells([ms.random_genome(600) for _ in range(20)])
    assert w.kinetics.N.size(2) == 128
    w.enzymatic_activity()
    assert torch.isfinite(w.cell_molecules).all()


def test_figure_sanity_checks_quick():
    """docs/figures.py: every supporting figure's sanity property holds (quick sizes, no plots)."""
    import importlib.util
    from pathlib import Path

    spec = importlib.util.spec_from_file_location("figures", Path(__file__).resolve().parents[1] / "docs" / "figures.py")
    fig = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(fig)
    check = fig.run(quick=True, plot=False)
    bad = [(n, d) for n, ok, d in check.results if not ok]
    assert not bad, bad


def test_demo_run_and_gif(tmp_path):
    """docs/run.py writes scalars, frames, checkpoints and the pickled world; docs/create_gif.py
    renders them; a checkpoint reloads into World.from_file."""
    import importlib.util
    import json
    from pathlib import Path

    root = Path(__file__).resolve().parents[1] / "docs"

    def load(name):
        spec = importlib.util.spec_from_file_location(name, root / f"{name}.py")
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        return mod

    run, gif = load("run"), load("create_gif")
    rundir = run.main(run._args(["--rundir", str(tmp_path / "r"), "--n-steps", "6", "--map-size", "32",
                                 "--init-n-cells", "60", "--check-every", "2", "--save-state", "--device", "cpu",
                                 "--seed", "1"]))
    lines = [json.loads(x) for x in open(rundir / "scalars.jsonl")]
    assert [x["step"] for x in lines] == [0, 2, 4] and "ATP" in lines[0]
    assert gif.create_gif([rundir, rundir], tmp_path / "c.gif") == 3
    import magicsoup_amd as ms

    w = ms.World.from_file(rundir=rundir)
    w.load_state(statedir=rundir / "step=4")
    assert w.n_cells == lines[-1]["n_cells"]
