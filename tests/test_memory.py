"""utils/memory.py: the HBM planner (CPU; the model is checked against live GPU worlds in
tests/test_gpu_kernels.py test_memory_model_matches_a_live_world)."""
from magicsoup_amd.utils import memory


def test_plan_fills_one_mi355x_past_the_old_pixel_cap():
    p = memory.plan(hbm_bytes=memory.MI355X_HBM, ranks=1, n_molecules=14, map_dtype="fp16", reserve=0.2)
    assert p["map_size"] % 256 == 0
    assert 0.7 <= p["fill"] <= 0.8
    assert p["per_rank"]["total"] <= p["budget_bytes"]
    bigger = memory.footprint(p["map_size"] + 256, 14, int(1e6 / 16384**2 * (p["map_size"] + 256) ** 2), "fp16")
    assert bigger["total"] > p["budget_bytes"]


def test_plan_is_not_capped_at_2_30_pixels():
    """64-bit map offsets in every kernel: a sparse world's rank holds more than 2^30 pixels."""
    p = memory.plan(ranks=1, cells_per_pixel=1e-4, reserve=0.2)
    assert p["map_size"] ** 2 > 1 << 31
    assert memory.plan(ranks=1, cells_per_pixel=1e-4, max_rank_pixels=1 << 30)["map_size"] ** 2 <= 1 << 30


def test_plan_per_rank_shrinks_with_ranks():
    one = memory.plan(ranks=1, reserve=0.2)
    eight = memory.plan(ranks=8, reserve=0.2)
    assert eight["map_size"] >= one["map_size"]
    assert eight["per_rank"]["cells_per_rank"] * 8 >= eight["cells"] - 8
    assert memory.plan(ranks=1, max_rank_pixels=1 << 30)["map_size"] ** 2 <= 1 << 30


def test_footprint_parts_scale():
    a = memory.footprint(4096, 14, 50_000, "fp32")
    b = memory.footprint(8192, 14, 50_000, "fp32")
    assert b["molecule_map"] == 4 * a["molecule_map"] and b["kinetics_rows"] == a["kinetics_rows"]
    h = memory.footprint(4096, 14, 50_000, "fp16")
    assert 2 * h["molecule_map"] == a["molecule_map"]
