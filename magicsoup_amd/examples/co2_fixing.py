"""Combined CO2-fixation chemistry (41 molecules, 46 reactions): Calvin cycle, Wood-Ljungdahl,
3-hydroxypropionate, reductive TCA, dicarboxylate/4-hydroxybutyrate and
3-hydroxypropionate/4-hydroxybutyrate pathways plus shared energy carriers.

Species, energies and reactions as in the reference ``python/magicsoup/examples/co2_fixing.py``.
As there, NADP has a different energy (130 kJ) than in the Wood-Ljungdahl example, so the two cannot
be imported into the same process (the Molecule registry rejects the conflict).
"""
from magicsoup_amd.examples._spec import chemistry, molecules

_FLOW = {"diffusivity": 1.0, "permeability": 1.0}
_M = molecules(
    [
        # shared carriers
        ("CO2", 10.0, _FLOW), ("NADPH", 200.0), ("NADP", 130.0), ("ATP", 100.0), ("ADP", 65.0),
        ("acetyl-CoA", 475.0), ("HS-CoA", 190.0), ("pyruvate", 330.0), ("G3P", 420.0), ("X", 50.0),
        ("E", 150.0),
        # Calvin cycle
        ("RuBP", 725.0), ("3PGA", 350.0), ("1,3BPG", 370.0), ("Ru5P", 695.0),
        # Wood-Ljungdahl
        ("methyl-FH4", 410.0), ("methylen-FH4", 355.0), ("formyl-FH4", 295.0), ("FH4", 200.0),
        ("formate", 70.0), ("CO", 75.0, _FLOW),
        # 3-hydroxypropionate
        ("malonyl-CoA", 495.0), ("propionyl-CoA", 675.0), ("methylmalonyl-CoA", 685.0),
        ("succinyl-CoA", 685.0), ("succinate", 485.0), ("fumarate", 415.0), ("malate", 415.0),
        ("malyl-CoA", 615.0), ("glyoxylate", 140.0), ("methylmalyl-CoA", 810.0), ("citramalyl-CoA", 810.0),
        # reductive TCA
        ("oxalacetate", 350.0), ("alpha-ketoglutarate", 540.0), ("isocitrate", 600.0), ("citrate", 600.0),
        # dicarboxylate / 4-hydroxybutyrate
        ("PEP", 350.0), ("SSA", 535.0), ("GHB", 600.0), ("hydroxybutyryl-CoA", 825.0), ("acetoacetyl-CoA", 760.0),
    ]
)

_COMMON = [
    "NADPH -> NADP",
    "ATP -> ADP",
    "2 ADP + E -> 2 ATP",
    "NADP + E -> NADPH",
    "G3P -> 8 X",
    "pyruvate -> 6 X",
    "acetyl-CoA -> HS-CoA + 5 X",
]
_CALVIN = [
    "RuBP + CO2 -> 2 3PGA",
    "3PGA + ATP -> 1,3BPG + ADP",
    "1,3BPG + NADPH -> G3P + NADP",
    "5 G3P -> 3 Ru5P",
    "Ru5P + ATP -> RuBP + ADP",
]
_WL = [
    "CO2 + NADPH -> formate + NADP",
    "formate + FH4 -> formyl-FH4",
    "formyl-FH4 + NADPH -> methylen-FH4 + NADP",
    "methylen-FH4 + NADPH -> methyl-FH4 + NADP",
    "CO2 + NADPH -> CO + NADP",
    "methyl-FH4 + CO + HS-CoA -> acetyl-CoA + FH4",
]
_HPROP = [
    "acetyl-CoA + CO2 -> malonyl-CoA",
    "malonyl-CoA + 3 NADPH -> propionyl-CoA + 3 NADP",
    "propionyl-CoA + CO2 -> methylmalonyl-CoA",
    "methylmalonyl-CoA -> succinyl-CoA",
    "succinyl-CoA -> succinate + HS-CoA",
    "succinate + NADP -> fumarate + NADPH",
    "fumarate -> malate",
    "malate + HS-CoA -> malyl-CoA",
    "malyl-CoA -> acetyl-CoA + glyoxylate",
    "propionyl-CoA + glyoxylate -> methylmalyl-CoA",
    "methylmalyl-CoA -> citramalyl-CoA",
    "citramalyl-CoA -> acetyl-CoA + pyruvate",
]
_RTCA = [
    "oxalacetate + NADPH -> malate + NADP",
    "malate -> fumarate",
    "fumarate + NADPH -> succinate + NADP",
    "succinate + HS-CoA -> succinyl-CoA",
    "succinyl-CoA + NADPH + CO2 -> alpha-ketoglutarate + HS-CoA + NADP",
    "alpha-ketoglutarate + CO2 + NADPH -> isocitrate + NADP",
    "isocitrate -> citrate",
    "citrate + HS-CoA -> oxalacetate + acetyl-CoA",
]
_DCHB = [
    "acetyl-CoA + CO2 + NADPH -> pyruvate + HS-CoA + NADP",
    "pyruvate + ATP -> PEP + ADP",
    "PEP + CO2 -> oxalacetate",
    "oxalacetate + NADPH -> malate + NADP",
    "malate -> fumarate",
    "fumarate + NADPH -> succinate + NADP",
    "succinate + HS-CoA -> succinyl-CoA",
    "succinyl-CoA + NADPH -> SSA + HS-CoA + NADP",
    "SSA + NADPH -> GHB + NADP",
    "GHB + HS-CoA -> hydroxybutyryl-CoA",
    "hydroxybutyryl-CoA + NADP -> acetoacetyl-CoA + NADPH",
    "acetoacetyl-CoA + HS-CoA -> 2 acetyl-CoA",
]
_HPHB = [
    "acetyl-CoA + CO2 -> malonyl-CoA",
    "malonyl-CoA + 3 NADPH -> propionyl-CoA + 3 NADP",
    "propionyl-CoA + CO2 -> methylmalonyl-CoA",
    "methylmalonyl-CoA -> succinyl-CoA",
    "succinyl-CoA + NADPH -> SSA + HS-CoA + NADP",
    "SSA + NADPH -> GHB + NADP",
    "GHB + HS-CoA -> hydroxybutyryl-CoA",
    "hydroxybutyryl-CoA + NADP -> acetoacetyl-CoA + NADPH",
    "acetoacetyl-CoA + HS-CoA -> 2 acetyl-CoA",
]

MOLECULES = list(_M.values())
CHEMISTRY = chemistry(list(_M), _COMMON + _CALVIN + _WL + _HPROP + _RTCA + _DCHB + _HPHB, _M)
REACTIONS = CHEMISTRY.reactions
