"""CPU tests of the host side: compiled model, RNG, workloads, and that libpnp.so loads and
exports every symbol include/pnp.h declares (no compute calls: there is no GPU here)."""
import ctypes as C
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "pnp.h")


def test_model_census(model):
    # SURVEY.md Appendix A
    assert (model.nq, model.nv, model.nu, model.nbody, model.njnt, model.nsite, model.nmocap, model.neq) == \
        (37, 33, 9, 20, 13, 7, 1, 1)
    coll = (model.geom_contype != 0) | (model.geom_conaffinity != 0)
    assert coll.sum() == 40
    assert np.allclose(model.body_mass[model.body_id("cube1")], 0.064)
    assert np.allclose(model.dof_armature[:9], 0.1) and np.allclose(model.dof_damping[:9], 1.0)
    assert np.allclose(model.jnt_range[3], [-3.0718, -0.0698])
    assert model.opt_timestep == 0.002 and model.opt_noslip_iterations == 3
    assert list(model.names_jnt[:9]) == [f"joint{i}" for i in range(1, 8)] + ["finger_joint1", "finger_joint2"]
    assert model.jnt_qposadr[model.joint_id("obj_joint")] == 30


@pytest.mark.skipif(not os.path.exists("/root/reference/panda_mujoco_gym/assets/shelf_pnp.xml"),
                    reason="reference MJCF only present in the build container")
def test_committed_model_matches_fresh_compile(model):
    from pnp_amd.mjcf import compile_xml
    fresh = compile_xml()
    for k, v in fresh.items():
        a = np.asarray(v)
        b = getattr(model, k) if not isinstance(getattr(model, k), np.ndarray) else getattr(model, k)
        if a.dtype.kind in "fi":
            np.testing.assert_allclose(np.asarray(b, a.dtype), a, err_msg=k)
        else:
            assert np.array_equal(np.asarray(b), a), k


def test_philox_known_answers():
    from pnp_amd import rng
    z = rng.philox4x32(np.zeros((1, 4), np.uint32), (0, 0))[0]
    assert [hex(x) for x in z] == ["0x6627e8d5", "0xe169c58d", "0xbc57ac4c", "0x9b00dbd8"]
    f = rng.philox4x32(np.full((1, 4), 0xFFFFFFFF, np.uint32), (0xFFFFFFFF, 0xFFFFFFFF))[0]
    assert [hex(x) for x in f] == ["0x408f276d", "0x41c83b0e", "0xa20bc7c6", "0x6d5451fd"]


def test_workload_is_shard_invariant(model):
    from pnp_amd import workloads
    full_q, full_d = workloads.ik_inputs(model, np.arange(256))
    for r in range(4):
        q, d = workloads.ik_inputs(model, np.arange(r * 64, (r + 1) * 64))
        assert np.array_equal(q, full_q[r * 64:(r + 1) * 64]) and np.array_equal(d, full_d[r * 64:(r + 1) * 64])
    lo, hi = model.jnt_range[:7, 0], model.jnt_range[:7, 1]
    span = hi - lo
    assert np.all(full_q >= lo + 0.05 * span - 1e-12) and np.all(full_q <= hi - 0.05 * span + 1e-12)
    assert np.all(np.abs(full_d) <= 0.02)


def _header_symbols():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int32_t|int64_t|const char\*)\s+(pnp_\w+)\s*\(", src, re.M)))


def test_library_loads_and_exports_header_symbols():
    from pnp_amd import _lib
    L = _lib.load()
    syms = _header_symbols()
    assert len(syms) >= 11
    for s in syms:
        assert hasattr(L, s), s
    assert set(syms) == set(_lib.EXPORTS)
    assert L.pnp_abi_version() == _lib.ABI_VERSION == 14
    from pnp_amd.model import PnpModelDesc
    assert L.pnp_model_desc_size() == C.sizeof(PnpModelDesc)


def test_library_rejects_bad_arguments_without_gpu():
    """Argument validation happens before any HIP call, so it is testable on the CPU."""
    from pnp_amd import _lib
    from pnp_amd.model import PnpIKParams
    L = _lib.load()
    rc = L.pnp_model_create(None, None)
    assert rc == -1 and b"null" in L.pnp_last_error()
    rc = L.pnp_ik_dls(None, 0, PnpIKParams(100, 1e-3, 1e-2, 0.1), None, None, None, None, None, None, None, 4, None)
    assert rc == -1 and b"bad argument" in L.pnp_last_error()


def test_tqc_entry_points_validate_without_gpu():
    """The fused learner's C entry points check shapes and pointers before any HIP call: the
    workspace size for train.py's shape (25 matrices [B][256] + 8 sums per 16-row slab), the
    parameter counts of the actor / critics, and refusals of unsupported shapes and null buffers."""
    from pnp_amd import _lib
    L = _lib.load()
    d = _lib.PnpTqcDesc()
    d.batch, d.obs_dim, d.act_dim, d.hidden, d.n_critics, d.n_quantiles, d.n_drop_per_net = 512, 25, 7, 256, 2, 25, 2
    assert L.pnp_tqc_workspace_floats(C.byref(d)) == 25 * 512 * 256 + (512 // 16) * 8
    na, nc = C.c_int32(), C.c_int32()
    assert L.pnp_tqc_param_counts(C.byref(na), C.byref(nc)) == 0
    # actor 25-256-256-256 + two 7-wide heads; critics 2 x (32-256-256-256-25)
    assert na.value == 25 * 256 + 256 + 2 * (256 * 256 + 256) + 2 * (256 * 7 + 7)
    assert nc.value == 2 * (32 * 256 + 256 + 2 * (256 * 256 + 256) + 256 * 25 + 25)
    d.hidden = 128                                   # not train.py's network
    assert L.pnp_tqc_workspace_floats(C.byref(d)) < 0 and b"unsupported" in L.pnp_last_error()
    d.hidden, d.batch = 256, 500                     # not a multiple of 16 rows
    assert L.pnp_tqc_workspace_floats(C.byref(d)) < 0
    d.batch = 512
    b = _lib.PnpTqcBatch()
    assert L.pnp_tqc_update(C.byref(d), C.byref(b), None, None) < 0   # no parameter pointers
    r = _lib.PnpTqcReplay()
    assert L.pnp_tqc_sample(C.byref(r), None, 512, None, None, None, None, None, None) < 0
    assert b"pnp_tqc_sample" in L.pnp_last_error()
    assert L.pnp_tqc_sample_draw(C.byref(r), 1, None, 512, None, None, None, None, None, None, None, None, None) < 0
    assert b"pnp_tqc_sample_draw" in L.pnp_last_error()


def test_product_package_never_imports_oracle():
    pkg = os.path.join(ROOT, "mujoco-panda-pnp_amd")
    for dp, _, fs in os.walk(pkg):
        for f in fs:
            if f.endswith((".py", ".hip", ".cpp", ".h")):
                txt = open(os.path.join(dp, f)).read()
                assert "import oracle" not in txt and "from oracle" not in txt and "liboracle" not in txt, f


def test_debug_layout_matches_header():
    """pnp_amd._lib.DBG mirrors the PNP_DBG_* offsets of include/pnp.h."""
    import re
    from pnp_amd import _lib
    hdr = open(os.path.join(ROOT, "include", "pnp.h")).read()
    defs = {k: int(v) for k, v in re.findall(r"#define PNP_DBG_(\w+) (\d+)", hdr)}
    assert defs == _lib.DBG


def test_model_check_builds_host_images_without_gpu(model):
    """pnp_model_check runs every host-side image builder pnp_model_create uploads (kinematics
    tables, both physics images: pair tables, broadphase body groups, hulls, the fp64 chain
    tables) with no HIP call -- the scene passes; descriptions past the compiled capacities or
    inconsistent ones are refused with a message.  (tools/asan_cpu_tests.sh runs this under
    ASan + UBSan.)"""
    from pnp_amd import _lib
    L = _lib.load()
    d = model.desc()
    assert L.pnp_model_check(C.byref(d)) == 0, L.pnp_last_error()
    assert L.pnp_model_check(None) == -1
    fresh = lambda: type(d).from_buffer_copy(model.desc())   # (desc() is cached: mutate copies)
    for field, value in (("nbody", 1000), ("nq", 10_000), ("nbody", 0)):
        bad = fresh()
        setattr(bad, field, value)
        assert L.pnp_model_check(C.byref(bad)) < 0, field
        assert L.pnp_last_error()
    bad = fresh()
    bad.nmeshvert = 100_000          # hulls past the step kernel's vertex capacity
    assert L.pnp_model_check(C.byref(bad)) == -3 and b"capacity" in L.pnp_last_error()
    # a hull whose vertex range runs past the vertex table: refused before any read of it
    import numpy as np
    vn = np.array(model.mesh_vertnum, np.int32).copy()
    vn[0] = model.nmeshvert + 5
    bad = fresh()
    bad.mesh_vertnum = vn.ctypes.data_as(C.POINTER(C.c_int32))
    assert L.pnp_model_check(C.byref(bad)) == -3 and b"mesh 0" in L.pnp_last_error()
    assert L.pnp_model_check(C.byref(model.desc())) == 0
