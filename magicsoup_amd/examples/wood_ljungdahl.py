"""Wood-Ljungdahl pathway chemistry (14 molecules, 6 reactions).

Same species, energies and reactions as the reference's benchmark / test chemistry
``python/magicsoup/examples/wood_ljungdahl.py`` (methyl and carbonyl branch, Co step skipped).
Energies in kJ/mol.
"""
from magicsoup_amd.examples._spec import chemistry, molecules

_M = molecules(
    [
        ("NADPH", 200.0),
        ("NADP", 100.0),
        ("ATP", 100.0),
        ("ADP", 70.0),
        ("methyl-FH4", 360.0),
        ("methylen-FH4", 300.0),
        ("formyl-FH4", 240.0),
        ("FH4", 200.0),
        ("formiat", 20.0),
        ("CO2", 10.0, {"diffusivity": 1.0, "permeability": 1.0}),
        ("Ni-ACS", 200.0),
        ("methyl-Ni-ACS", 300.0),
        ("HS-CoA", 200.0),
        ("acetyl-CoA", 260.0),
    ]
)

_EQUATIONS = [
    "CO2 + NADPH -> formiat + NADP",
    "formiat + FH4 + ATP -> formyl-FH4 + ADP",
    "formyl-FH4 + NADPH -> methylen-FH4 + NADP",
    "methylen-FH4 + NADPH -> methyl-FH4 + NADP",
    "methyl-FH4 + Ni-ACS -> FH4 + methyl-Ni-ACS",
    "methyl-Ni-ACS + CO2 + HS-CoA -> Ni-ACS + acetyl-CoA",
]

MOLECULES = list(_M.values())
CHEMISTRY = chemistry(list(_M), _EQUATIONS, _M)
REACTIONS = CHEMISTRY.reactions
