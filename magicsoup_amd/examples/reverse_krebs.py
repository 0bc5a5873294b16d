"""Reverse Krebs cycle chemistry (15 molecules, 8 reactions); reference examples/reverse_krebs.py."""
from magicsoup_amd.examples._spec import chemistry, molecules

_M = molecules(
    [
        ("NADPH", 200.0),
        ("NADP", 100.0),
        ("ATP", 100.0),
        ("ADP", 70.0),
        ("CO2", 10.0, {"diffusivity": 1.0, "permeability": 1.0}),
        ("oxalalcetate", 200.0),
        ("malate", 250.0),
        ("fumarate", 240.0),
        ("sucinate", 300.0),
        ("sucinyl-CoA", 500.0),
        ("oxoglutarate", 300.0),
        ("isocitrate", 350.0),
        ("citrate", 340.0),
        ("HS-CoA", 200.0),
        ("acetyl-CoA", 260.0),
    ]
)
_EQUATIONS = [
    "oxalalcetate + NADPH -> malate + NADP",
    "malate -> fumarate",
    "fumarate + NADPH -> sucinate + NADP",
    "sucinate + ATP + HS-CoA -> sucinyl-CoA + ADP",
    "sucinyl-CoA + CO2 -> oxoglutarate + HS-CoA",
    "oxoglutarate + CO2 + NADPH -> isocitrate + NADP",
    "isocitrate -> citrate",
    "citrate + HS-CoA -> acetyl-CoA + oxalalcetate",
]
MOLECULES = list(_M.values())
CHEMISTRY = chemistry(list(_M), _EQUATIONS, _M)
REACTIONS = CHEMISTRY.reactions
