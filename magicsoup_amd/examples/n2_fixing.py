"""Nitrogen fixation chemistry (10 molecules, 2 reactions); reference examples/n2_fixing.py."""
from magicsoup_amd.examples._spec import chemistry, molecules

_M = molecules(
    [
        ("NADPH", 200.0),
        ("NADP", 100.0),
        ("ATP", 100.0),
        ("ADP", 70.0),
        ("ammonia", 10.0),
        ("glutamate", 200.0),
        ("glutamine", 220.0),
        ("oxalalcetate", 200.0),
        ("HS-CoA", 200.0),
        ("acetyl-CoA", 260.0),
    ]
)
_EQUATIONS = [
    "glutamate + ATP + ammonia -> ADP + glutamine",
    "oxalalcetate + glutamine + NADPH -> 2 glutamate + NADP",
]
MOLECULES = list(_M.values())
CHEMISTRY = chemistry(list(_M), _EQUATIONS, _M)
REACTIONS = CHEMISTRY.reactions
