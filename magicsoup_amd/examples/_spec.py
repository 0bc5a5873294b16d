"""Tiny reaction-equation DSL used to declare the example chemistries.

``"2 NADPH + CO2 -> formate + NADP"`` becomes ``([NADPH, NADPH, CO2], [formate, NADP])`` with the
molecules looked up in a name -> Molecule table.
"""
from __future__ import annotations

from magicsoup_amd.models.containers import Chemistry, Molecule


def molecules(table: list[tuple]) -> dict[str, Molecule]:
    """``[(name, energy_kJ, {kwargs}?), ...]`` -> {name: Molecule}; energies given in kJ/mol."""
    out = {}
    for row in table:
        name, kj = row[0], row[1]
        kw = row[2] if len(row) > 2 else {}
        out[name] = Molecule(name, kj * 1e3, **kw)
    return out


def _side(text: str, mols: dict[str, Molecule]) -> list[Molecule]:
    out: list[Molecule] = []
    for term in (t.strip() for t in text.split(" + ")):
        parts = term.split(" ", 1)
        if len(parts) == 2 and parts[0].isdigit():
            out += [mols[parts[1].strip()]] * int(parts[0])
        else:
            out.append(mols[term])
    return out


def reaction(eq: str, mols: dict[str, Molecule]) -> tuple[list[Molecule], list[Molecule]]:
    lhs, rhs = eq.split("->")
    return _side(lhs.strip(), mols), _side(rhs.strip(), mols)


def chemistry(mol_names: list[str], equations: list[str], mols: dict[str, Molecule]) -> Chemistry:
    return Chemistry(molecules=[mols[n] for n in mol_names], reactions=[reaction(e, mols) for e in equations])
