"""Behaviour-tree semantics of pnp_amd/bt.py (py_trees 2.2.2 restated for the reference's
behavior_tree/ package; py_trees is absent here): Behaviour.tick's initialise / update / terminate
order, Sequence(memory=True) handing a succeeded child's tick to the next child and restarting
after it finished, Retry, and build_pnp_tree's shape (trees/pnp_tree.py)."""
from pnp_amd import bt


class Rec(bt.Behaviour):
    def __init__(self, name, script, log):
        super().__init__(name)
        self.script, self.log, self.i = list(script), log, 0

    def initialise(self):
        self.log.append(("init", self.name))

    def update(self):
        st = self.script[min(self.i, len(self.script) - 1)]
        self.i += 1
        self.log.append(("update", self.name, st))
        return st

    def terminate(self, new_status):
        self.log.append(("term", self.name, new_status))


S, R, F = bt.Status.SUCCESS, bt.Status.RUNNING, bt.Status.FAILURE


def test_behaviour_tick_order():
    log = []
    b = Rec("a", [R, S], log)
    assert b.tick() == R and b.tick() == S
    assert log == [("init", "a"), ("update", "a", R), ("update", "a", S), ("term", "a", S)]
    assert b.status == S


def test_sequence_memory_hands_the_tick_on():
    log = []
    a, b, c = Rec("a", [S], log), Rec("b", [R, S], log), Rec("c", [S], log)
    seq = bt.Sequence("s", [a, b, c])
    assert seq.tick() == R                      # a succeeds, b starts in the same tick
    assert [e[:2] for e in log] == [("init", "a"), ("update", "a"), ("term", "a"), ("init", "b"), ("update", "b")]
    log.clear()
    assert seq.tick() == S                      # b resumes (memory), c runs in the same tick
    assert ("init", "a") not in log and ("update", "c", S) in log
    log.clear()
    a.script, b.script, c.script = [R], [S], [S]
    a.i = b.i = c.i = 0
    assert seq.tick() == R                      # finished sequence restarts from the first child
    assert ("term", "a", bt.Status.INVALID) in log and ("init", "a") in log


def test_sequence_failure_and_retry():
    log = []
    flaky = Rec("p", [F, S], log)
    r = bt.Retry("r", flaky, num_failures=3)
    assert r.tick() == R                        # first failure: retried
    assert r.tick() == S
    log2 = []
    r2 = bt.Retry("r2", Rec("q", [F], log2), num_failures=1)
    assert r2.tick() == F


def test_build_pnp_tree_shape():
    class Env:
        action_space = type("A", (), {"low": [0] * 7})()
    tasks = [{"obj_meta": {"id": 1, "delta_q": [0, 0, 0, 1], "approach_wpt1": 0, "obj_pos": 0, "approach_wpt2": 0},
              "place_meta": {}} for _ in range(3)]
    t = bt.build_pnp_tree(Env(), tasks, retry_pick=1)
    assert len(t.root.children) == 3
    kinds = [[type(c).__name__ for c in sub.children] for sub in t.root.children]
    assert kinds == [["PickNode", "PlaceNode", "HomeNode"]] * 3
    t3 = bt.build_pnp_tree(Env(), tasks[:1], retry_pick=3)
    assert type(t3.root.children[0].children[0]).__name__ == "Retry"


def test_sequence_reset_stops_a_retried_child():
    """py_trees Decorator.stop: when a Sequence restarts (its children stopped with INVALID), a
    Retry stops its decorated child too, so the child's status and state do not stay stale; a child
    still RUNNING when the decorator itself finishes is stopped as well."""
    log = []
    child = Rec("pick", [R], log)
    seq = bt.Sequence("s", [bt.Retry("r", child, num_failures=3)])
    assert seq.tick() == R and child.status == R
    seq.status = bt.Status.INVALID              # parent interrupted: the next tick restarts it
    log.clear()
    seq.tick()
    assert ("term", "pick", bt.Status.INVALID) in log
    assert log.index(("term", "pick", bt.Status.INVALID)) < log.index(("init", "pick"))
    log2 = []
    c2 = Rec("c", [R], log2)
    r = bt.Retry("r", c2, num_failures=2)
    r.tick()
    r.stop(bt.Status.FAILURE)                   # decorator ends while the child still runs
    assert c2.status == bt.Status.INVALID and ("term", "c", bt.Status.INVALID) in log2
