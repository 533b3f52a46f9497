"""MJCF compiler for the Panda shelf pick-and-place scene.

Turns the two MJCF files the reference loads (``assets/shelf_pnp.xml`` which includes
``assets/panda_mocap.xml``; loaded at reference ``envs/panda_env.py:108`` through
``MjModel.from_xml_path``) into flat, MjModel-style constant arrays that the HIP engine copies to
the device once per model (``pnp_model_create`` in ``include/pnp.h``).

Only the MJCF features these two files use are implemented: nested ``<default>`` classes with
``childclass``/``class`` resolution, ``<include>``, bodies with ``pos``/``quat``, ``mocap``,
``<inertial>`` (``fullinertia``/``diaginertia``) or geom-derived inertia (box/sphere, density
1000), hinge/slide/free joints, geoms (collision meshes are reduced to convex hulls, the form
MuJoCo collides them in), sites, ``general`` actuators with affine bias, a weld equality and the
``<option>`` block.  Upstream semantics restated from MuJoCo 2.3.3's compiler (``user_model.cc``,
``user_objects.cc``): quaternions are normalised, ``autolimits`` sets ``limited`` when a range is
given, body order is depth-first document order with the included worldbody first.

This runs where ``/root/reference`` exists; its output (``data/panda_shelf.npz``) is committed,
so the GPU box never reads the reference.  ``python -m pnp_amd.mjcf`` regenerates it.
"""
from __future__ import annotations

import os
import struct
import xml.etree.ElementTree as ET
from dataclasses import dataclass, field

import numpy as np

# MuJoCo enum values (mjtJoint, mjtGeom) so the arrays read like MjModel fields.
JNT_FREE, JNT_BALL, JNT_SLIDE, JNT_HINGE = 0, 1, 2, 3
GEOM_PLANE, GEOM_HFIELD, GEOM_SPHERE, GEOM_CAPSULE, GEOM_ELLIPSOID, GEOM_CYLINDER, GEOM_BOX, GEOM_MESH = range(8)
_GEOM_TYPES = {"plane": GEOM_PLANE, "sphere": GEOM_SPHERE, "capsule": GEOM_CAPSULE,
               "ellipsoid": GEOM_ELLIPSOID, "cylinder": GEOM_CYLINDER, "box": GEOM_BOX, "mesh": GEOM_MESH}
_JNT_TYPES = {"free": JNT_FREE, "ball": JNT_BALL, "slide": JNT_SLIDE, "hinge": JNT_HINGE}

# MuJoCo built-in defaults (the "main" class before any user override).
_BUILTIN = {
    "joint": {"type": "hinge", "pos": "0 0 0", "axis": "0 0 1", "armature": "0", "damping": "0",
              "stiffness": "0", "frictionloss": "0"},
    "geom": {"type": "sphere", "pos": "0 0 0", "quat": "1 0 0 0", "contype": "1", "conaffinity": "1",
             "condim": "3", "group": "0", "friction": "1 0.005 0.0001", "solref": "0.02 1",
             "solimp": "0.9 0.95 0.001 0.5 2", "margin": "0", "gap": "0", "priority": "0",
             "density": "1000", "size": "0 0 0"},
    "site": {"pos": "0 0 0", "quat": "1 0 0 0"},
    "general": {"gear": "1 0 0 0 0 0", "gainprm": "1 0 0", "biasprm": "0 0 0", "dyntype": "none",
                "gaintype": "fixed", "biastype": "none"},
}


def _vec(s, n=None):
    v = np.array([float(x) for x in s.split()], dtype=np.float64)
    if n is not None and v.size < n:
        v = np.concatenate([v, np.zeros(n - v.size)])
    return v


def _quat_normalize(q):
    q = np.asarray(q, np.float64)
    return q / np.linalg.norm(q)


def quat2mat(q):
    """wxyz unit quaternion -> row-major 3x3 (MuJoCo ``mju_quat2Mat`` convention)."""
    w, x, y, z = q
    return np.array([
        [1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
        [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
        [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])


def mat2quat(R):
    """Rotation matrix -> wxyz quaternion (w >= 0)."""
    tr = np.trace(R)
    if tr > 0:
        s = np.sqrt(tr + 1.0) * 2
        q = [0.25 * s, (R[2, 1] - R[1, 2]) / s, (R[0, 2] - R[2, 0]) / s, (R[1, 0] - R[0, 1]) / s]
    elif R[0, 0] > R[1, 1] and R[0, 0] > R[2, 2]:
        s = np.sqrt(1.0 + R[0, 0] - R[1, 1] - R[2, 2]) * 2
        q = [(R[2, 1] - R[1, 2]) / s, 0.25 * s, (R[0, 1] + R[1, 0]) / s, (R[0, 2] + R[2, 0]) / s]
    elif R[1, 1] > R[2, 2]:
        s = np.sqrt(1.0 + R[1, 1] - R[0, 0] - R[2, 2]) * 2
        q = [(R[0, 2] - R[2, 0]) / s, (R[0, 1] + R[1, 0]) / s, 0.25 * s, (R[1, 2] + R[2, 1]) / s]
    else:
        s = np.sqrt(1.0 + R[2, 2] - R[0, 0] - R[1, 1]) * 2
        q = [(R[1, 0] - R[0, 1]) / s, (R[0, 2] + R[2, 0]) / s, (R[1, 2] + R[2, 1]) / s, 0.25 * s]
    q = np.array(q)
    if q[0] < 0:
        q = -q
    return _quat_normalize(q)


def _principal_inertia(full):
    """Full inertia tensor -> (diag, iquat) with a right-handed principal frame."""
    w, V = np.linalg.eigh(full)
    order = np.argsort(-w)           # MuJoCo keeps eigenvalues in decreasing order
    w, V = w[order], V[:, order]
    if np.linalg.det(V) < 0:
        V[:, 2] = -V[:, 2]
    return w, mat2quat(V)


# ----------------------------------------------------------------------------- mesh loading
def _load_mesh_vertices(path):
    if path.lower().endswith(".stl"):
        with open(path, "rb") as f:
            data = f.read()
        n = struct.unpack_from("<I", data, 80)[0]
        if 84 + 50 * n == len(data):
            tri = np.frombuffer(data, dtype=np.dtype([("n", "<f4", 3), ("v", "<f4", (3, 3)), ("a", "<u2")]),
                                count=n, offset=84)
            return tri["v"].reshape(-1, 3).astype(np.float64)
        verts = [[float(t) for t in ln.split()[1:4]] for ln in data.decode().splitlines()
                 if ln.strip().startswith("vertex")]
        return np.array(verts, np.float64)
    verts = []
    with open(path) as f:
        for ln in f:
            if ln.startswith("v "):
                verts.append([float(t) for t in ln.split()[1:4]])
    return np.array(verts, np.float64)


def _convex_hull(verts):
    from scipy.spatial import ConvexHull
    v = np.unique(np.round(verts, 9), axis=0)
    hull = ConvexHull(v)
    hv = v[hull.vertices]
    return hv


def _hull_centroid(hv):
    """Volume centroid of the convex hull of hv: tetrahedra from an interior point (the vertex
    mean) to every hull facet."""
    from scipy.spatial import ConvexHull
    hull = ConvexHull(hv)
    c0 = hv.mean(0)
    vol, cen = 0.0, np.zeros(3)
    for tri in hull.simplices:
        a, b, c = hv[tri]
        w = abs(np.dot(a - c0, np.cross(b - c0, c - c0))) / 6.0
        vol += w
        cen += w * (a + b + c + c0) / 4.0
    return cen / vol


# ----------------------------------------------------------------------------- parser
@dataclass
class _Class:
    name: str
    parent: "_Class | None"
    attrs: dict = field(default_factory=dict)   # element tag -> attr dict (own overrides)

    def resolve(self, tag):
        chain = []
        c = self
        while c is not None:
            chain.append(c)
            c = c.parent
        out = dict(_BUILTIN.get(tag, {}))
        for c in reversed(chain):
            out.update(c.attrs.get(tag, {}))
        return out


class MJCFCompiler:
    def __init__(self, xml_path):
        self.xml_path = os.path.abspath(xml_path)
        self.dir = os.path.dirname(self.xml_path)
        self.classes = {"main": _Class("main", None)}
        self.meshes = {}
        self.meshdir = ""
        self.option = {"timestep": 0.002, "integrator": "Euler", "noslip_iterations": 0,
                       "cone": "pyramidal", "gravity": [0, 0, -9.81], "multiccd": 0, "warmstart": 1,
                       "iterations": 100, "tolerance": 1e-8, "solver": "Newton", "noslip_tolerance": 1e-6}
        self.autolimits = True
        root = self._expand(ET.parse(self.xml_path).getroot(), self.dir)
        self.root = root

    # merge <include> files in place (their <mujoco> children are spliced in)
    def _expand(self, elem, base):
        new_children = []
        for ch in list(elem):
            if ch.tag == "include":
                inc = ET.parse(os.path.join(base, ch.get("file"))).getroot()
                inc = self._expand(inc, base)
                new_children.extend(list(inc))
            else:
                new_children.append(self._expand(ch, base))
        for ch in list(elem):
            elem.remove(ch)
        for ch in new_children:
            elem.append(ch)
        return elem

    def _parse_defaults(self, elem, parent):
        for d in elem.findall("default"):
            name = d.get("class", "main")
            cls = self.classes.get(name) if name == "main" else None
            if cls is None:
                cls = _Class(name, parent)
                self.classes[name] = cls
            for ch in d:
                if ch.tag == "default":
                    continue
                cls.attrs.setdefault(ch.tag, {}).update(ch.attrib)
            self._parse_defaults(d, cls)

    def compile(self):
        r = self.root
        for c in r.findall("compiler"):
            self.meshdir = c.get("meshdir", self.meshdir)
            self.autolimits = c.get("autolimits", "true") == "true"
            assert c.get("angle", "radian") == "radian"
        for o in r.findall("option"):
            for k in ("timestep", "tolerance", "noslip_tolerance"):
                if o.get(k):
                    self.option[k] = float(o.get(k))
            for k in ("noslip_iterations", "iterations"):
                if o.get(k):
                    self.option[k] = int(o.get(k))
            for k in ("integrator", "cone", "solver"):
                if o.get(k):
                    self.option[k] = o.get(k)
            for fl in o.findall("flag"):
                for k, v in fl.attrib.items():
                    self.option[k] = 1 if v == "enable" else 0
        for d in r.findall("default"):
            # top-level <default> is the "main" class (possibly with nested classes)
            name = d.get("class", "main")
            cls = self.classes["main"] if name == "main" else _Class(name, self.classes["main"])
            self.classes[name] = cls
            for ch in d:
                if ch.tag != "default":
                    cls.attrs.setdefault(ch.tag, {}).update(ch.attrib)
            self._parse_defaults(d, cls)
        for a in r.findall("asset"):
            for m in a.findall("mesh"):
                f = m.get("file")
                name = m.get("name", os.path.splitext(os.path.basename(f))[0])
                self.meshes[name] = os.path.join(self.dir, self.meshdir, f)

        M = _ModelBuilder(self)
        world = M.add_body(None, "world", {}, None)
        for wb in r.findall("worldbody"):
            M.walk(wb, world, "main", is_world=True)
        for act in r.findall("actuator"):
            for g in act:
                M.add_actuator(g)
        for eq in r.findall("equality"):
            for w in eq:
                M.add_equality(w)
        return M.finish()


class _ModelBuilder:
    def __init__(self, comp: MJCFCompiler):
        self.c = comp
        self.bodies, self.joints, self.geoms, self.sites = [], [], [], []
        self.actuators, self.eqs = [], []
        self.body_names, self.joint_names, self.geom_names, self.site_names = [], [], [], []

    def _attrs(self, elem, tag, childclass):
        cls = self.c.classes[elem.get("class", childclass)]
        a = cls.resolve(tag)
        a.update({k: v for k, v in elem.attrib.items() if k != "class"})
        return a

    def add_body(self, parent, name, attrib, elem):
        bid = len(self.bodies)
        b = {"name": name, "parent": parent if parent is not None else 0,
             "pos": _vec(attrib.get("pos", "0 0 0")),
             "quat": _quat_normalize(_vec(attrib.get("quat", "1 0 0 0"))),
             "mocap": attrib.get("mocap", "false") == "true", "inertial": None, "geoms": [],
             "joints": []}
        if elem is not None:
            ine = elem.find("inertial")
            if ine is not None:
                b["inertial"] = ine.attrib
        self.bodies.append(b)
        self.body_names.append(name)
        return bid

    def walk(self, elem, bid, childclass, is_world=False):
        for ch in elem:
            if ch.tag == "body":
                cc = ch.get("childclass", childclass)
                nb = self.add_body(bid, ch.get("name", f"body{len(self.bodies)}"), ch.attrib, ch)
                self._body_elems(ch, nb, cc)
                self.walk(ch, nb, cc)
        if is_world:
            self._body_elems(elem, bid, childclass)

    def _body_elems(self, elem, bid, cc):
        for ch in elem:
            if ch.tag == "joint":
                a = self._attrs(ch, "joint", cc)
                self.joints.append({"body": bid, **a})
                self.joint_names.append(ch.get("name", f"joint{len(self.joints)}"))
                self.bodies[bid]["joints"].append(len(self.joints) - 1)
            elif ch.tag == "freejoint":
                self.joints.append({"body": bid, "type": "free", "pos": "0 0 0", "axis": "0 0 1",
                                    "armature": "0", "damping": "0"})
                self.joint_names.append(ch.get("name", f"joint{len(self.joints)}"))
                self.bodies[bid]["joints"].append(len(self.joints) - 1)
            elif ch.tag == "geom":
                a = self._attrs(ch, "geom", cc)
                self.geoms.append({"body": bid, **a})
                self.geom_names.append(ch.get("name", ""))
                self.bodies[bid]["geoms"].append(len(self.geoms) - 1)
            elif ch.tag == "site":
                a = self._attrs(ch, "site", cc)
                self.sites.append({"body": bid, **a})
                self.site_names.append(ch.get("name", ""))

    def add_actuator(self, g):
        a = self._attrs(g, g.tag, "main")
        a["_tag"] = g.tag
        self.actuators.append(a)

    def add_equality(self, w):
        a = dict(w.attrib)
        a["_tag"] = w.tag
        self.eqs.append(a)

    # ------------------------------------------------------------------ finish
    def finish(self):
        nb = len(self.bodies)
        # MuJoCo renumbers sites/geoms/joints in body order (bodies are already depth-first).
        jorder = sorted(range(len(self.joints)), key=lambda j: (self.joints[j]["body"], j))
        gorder = sorted(range(len(self.geoms)), key=lambda g: (self.geoms[g]["body"], g))
        sorder = sorted(range(len(self.sites)), key=lambda s: (self.sites[s]["body"], s))
        joints = [self.joints[j] for j in jorder]
        jnames = [self.joint_names[j] for j in jorder]
        geoms = [self.geoms[g] for g in gorder]
        gnames = [self.geom_names[g] for g in gorder]
        sites = [self.sites[s] for s in sorder]
        snames = [self.site_names[s] for s in sorder]

        out = {}
        # ---- joints / dofs
        nj = len(joints)
        jnt_type = np.zeros(nj, np.int32)
        jnt_qposadr = np.zeros(nj, np.int32)
        jnt_dofadr = np.zeros(nj, np.int32)
        jnt_bodyid = np.zeros(nj, np.int32)
        jnt_pos = np.zeros((nj, 3))
        jnt_axis = np.zeros((nj, 3))
        jnt_range = np.zeros((nj, 2))
        jnt_limited = np.zeros(nj, np.int32)
        jnt_solref = np.tile([0.02, 1.0], (nj, 1))          # solreflimit default
        jnt_solimp = np.tile([0.9, 0.95, 0.001, 0.5, 2.0], (nj, 1))   # solimplimit default
        jnt_margin = np.zeros(nj)
        dof_armature, dof_damping, dof_jntid, dof_bodyid = [], [], [], []
        qpos0 = []
        nq = nv = 0
        for j, a in enumerate(joints):
            t = _JNT_TYPES[a.get("type", "hinge")]
            jnt_type[j] = t
            jnt_bodyid[j] = a["body"]
            jnt_qposadr[j] = nq
            jnt_dofadr[j] = nv
            jnt_pos[j] = _vec(a.get("pos", "0 0 0"))
            ax = _vec(a.get("axis", "0 0 1"))
            jnt_axis[j] = ax / np.linalg.norm(ax)
            if "solreflimit" in a:
                jnt_solref[j] = _vec(a["solreflimit"])
            if "solimplimit" in a:
                si = _vec(a["solimplimit"])
                jnt_solimp[j] = np.concatenate([si, jnt_solimp[j][si.size:]])
            jnt_margin[j] = float(a.get("margin", 0))
            if t != JNT_FREE and "range" in a:
                jnt_range[j] = _vec(a["range"])
                lim = a.get("limited", "auto")
                jnt_limited[j] = 1 if (lim == "true" or (lim == "auto" and self.c.autolimits)) else 0
            ndof = {JNT_FREE: 6, JNT_BALL: 3}.get(t, 1)
            nqj = {JNT_FREE: 7, JNT_BALL: 4}.get(t, 1)
            if t == JNT_FREE:
                b = self.bodies[a["body"]]
                qpos0 += list(b["pos"]) + list(b["quat"])
            elif t == JNT_BALL:
                qpos0 += [1, 0, 0, 0]
            else:
                qpos0 += [float(a.get("ref", 0.0))]
            for _ in range(ndof):
                dof_armature.append(float(a.get("armature", 0)))
                dof_damping.append(float(a.get("damping", 0)))
                dof_jntid.append(j)
                dof_bodyid.append(a["body"])
            nq += nqj
            nv += ndof
        # ---- bodies
        body_parentid = np.array([b["parent"] for b in self.bodies], np.int32)
        body_parentid[0] = 0
        body_pos = np.array([b["pos"] for b in self.bodies])
        body_quat = np.array([b["quat"] for b in self.bodies])
        body_jntadr = -np.ones(nb, np.int32)
        body_jntnum = np.zeros(nb, np.int32)
        for j in range(nj):
            bj = jnt_bodyid[j]
            if body_jntadr[bj] < 0:
                body_jntadr[bj] = j
            body_jntnum[bj] += 1
        body_dofadr = -np.ones(nb, np.int32)
        body_dofnum = np.zeros(nb, np.int32)
        for d, bj in enumerate(dof_bodyid):
            if body_dofadr[bj] < 0:
                body_dofadr[bj] = d
            body_dofnum[bj] += 1
        body_mocapid = -np.ones(nb, np.int32)
        nmocap = 0
        for i, b in enumerate(self.bodies):
            if b["mocap"]:
                body_mocapid[i] = nmocap
                nmocap += 1
        # weldid: nearest ancestor (incl. self) with a joint, 0 = welded to world
        body_weldid = np.zeros(nb, np.int32)
        for i in range(1, nb):
            body_weldid[i] = i if body_jntnum[i] > 0 else body_weldid[body_parentid[i]]
        body_rootid = np.zeros(nb, np.int32)
        for i in range(1, nb):
            body_rootid[i] = i if body_parentid[i] == 0 else body_rootid[body_parentid[i]]
        # inertia
        body_mass = np.zeros(nb)
        body_ipos = np.zeros((nb, 3))
        body_iquat = np.tile([1.0, 0, 0, 0], (nb, 1))
        body_inertia = np.zeros((nb, 3))
        for i, b in enumerate(self.bodies):
            if i == 0:
                continue
            if b["inertial"] is not None:
                ia = b["inertial"]
                body_mass[i] = float(ia["mass"])
                body_ipos[i] = _vec(ia.get("pos", "0 0 0"))
                if "fullinertia" in ia:
                    f = _vec(ia["fullinertia"])
                    full = np.array([[f[0], f[3], f[4]], [f[3], f[1], f[5]], [f[4], f[5], f[2]]])
                    if "quat" in ia:
                        Rq = quat2mat(_quat_normalize(_vec(ia["quat"])))
                        full = Rq @ full @ Rq.T
                    body_inertia[i], body_iquat[i] = _principal_inertia(full)
                else:
                    body_inertia[i] = _vec(ia["diaginertia"])
                    body_iquat[i] = _quat_normalize(_vec(ia.get("quat", "1 0 0 0")))
            else:
                m_tot, com, I_tot = 0.0, np.zeros(3), np.zeros((3, 3))
                parts = []
                for gi in b["geoms"]:
                    g = self.geoms[gi]
                    t = _GEOM_TYPES[g.get("type", "sphere")]
                    size = _vec(g.get("size", "0 0 0"), 3)
                    rho = float(g.get("density", 1000))
                    gp = _vec(g.get("pos", "0 0 0"))
                    gq = _quat_normalize(_vec(g.get("quat", "1 0 0 0")))
                    if t == GEOM_BOX:
                        m = rho * 8 * size[0] * size[1] * size[2]
                        I = m / 3 * np.diag([size[1] ** 2 + size[2] ** 2, size[0] ** 2 + size[2] ** 2,
                                             size[0] ** 2 + size[1] ** 2])
                    elif t == GEOM_SPHERE:
                        m = rho * 4.0 / 3.0 * np.pi * size[0] ** 3
                        I = 0.4 * m * size[0] ** 2 * np.eye(3)
                    else:
                        continue   # mocap / visual meshes: not needed (their bodies have <inertial>)
                    Rg = quat2mat(gq)
                    parts.append((m, gp, Rg @ I @ Rg.T))
                    m_tot += m
                    com += m * gp
                if m_tot > 0:
                    com /= m_tot
                    for m, gp, I in parts:
                        d = gp - com
                        I_tot += I + m * (np.dot(d, d) * np.eye(3) - np.outer(d, d))
                    body_mass[i] = m_tot
                    body_ipos[i] = com
                    body_inertia[i], body_iquat[i] = _principal_inertia(I_tot)
        # ---- geoms (collision-relevant fields)
        ng = len(geoms)
        geom_type = np.zeros(ng, np.int32)
        geom_bodyid = np.zeros(ng, np.int32)
        geom_contype = np.zeros(ng, np.int32)
        geom_conaffinity = np.zeros(ng, np.int32)
        geom_condim = np.zeros(ng, np.int32)
        geom_priority = np.zeros(ng, np.int32)
        geom_size = np.zeros((ng, 3))
        geom_pos = np.zeros((ng, 3))
        geom_quat = np.zeros((ng, 4))
        geom_friction = np.zeros((ng, 3))
        geom_solref = np.zeros((ng, 2))
        geom_solimp = np.zeros((ng, 5))
        geom_margin = np.zeros(ng)
        geom_gap = np.zeros(ng)
        geom_dataid = -np.ones(ng, np.int32)
        geom_solmix = np.ones(ng)
        geom_rbound = np.zeros(ng)
        mesh_names, mesh_vert, mesh_vertadr, mesh_vertnum, mesh_center = [], [], [], [], []
        for k, g in enumerate(geoms):
            t = _GEOM_TYPES[g.get("type", "sphere")]
            geom_type[k] = t
            geom_bodyid[k] = g["body"]
            geom_contype[k] = int(g.get("contype", 1))
            geom_conaffinity[k] = int(g.get("conaffinity", 1))
            geom_condim[k] = int(g.get("condim", 3))
            geom_priority[k] = int(g.get("priority", 0))
            geom_size[k] = _vec(g.get("size", "0 0 0"), 3)[:3]
            geom_pos[k] = _vec(g.get("pos", "0 0 0"))
            geom_quat[k] = _quat_normalize(_vec(g.get("quat", "1 0 0 0")))
            fr = _vec(g.get("friction", "1 0.005 0.0001"))
            if fr.size < 3:
                fr = np.concatenate([fr, _vec("1 0.005 0.0001")[fr.size:]])
            geom_friction[k] = fr
            geom_solref[k] = _vec(g.get("solref", "0.02 1"))
            si = _vec(g.get("solimp", "0.9 0.95 0.001 0.5 2"))
            geom_solimp[k] = np.concatenate([si, _vec("0.9 0.95 0.001 0.5 2")[si.size:]])
            geom_margin[k] = float(g.get("margin", 0))
            geom_gap[k] = float(g.get("gap", 0))
            geom_solmix[k] = float(g.get("solmix", 1))
            collidable = geom_contype[k] != 0 or geom_conaffinity[k] != 0
            if t == GEOM_MESH and collidable:
                # MuJoCo's mesh compiler moves a mesh into its own frame at the mesh's centre of mass
                # and shifts the geom frame by the same offset (mjCMesh / mjCGeom: geom pos += quat
                # * mesh pos): the geom centre -- MPR's interior point -- then lies inside the hull.
                # Here the centre is the hull's volume centroid (the collision shape is the hull;
                # for a convex mesh the two coincide).  Without it the finger meshes' frames sit
                # outside their hulls, and MPR reported ~5 cm of phantom penetration between two
                # closed fingers whose hulls are 3 mm apart.
                mname = g["mesh"]
                if mname not in mesh_names:
                    hv = _convex_hull(_load_mesh_vertices(self.c.meshes[mname]))
                    cen = _hull_centroid(hv)
                    # stored in single precision like MuJoCo's mjModel.mesh_vert (float*): the
                    # recentred vertices rounded once, so the fp64 oracle and the fp32 kernels'
                    # images hold the same values (unrounded, the fp32 image's own rounding tilted
                    # two finger faces in contact by ~1e-7 rad against the oracle's)
                    hv = (hv - cen).astype(np.float32).astype(np.float64)
                    mesh_vertadr.append(sum(len(v) for v in mesh_vert))
                    mesh_vertnum.append(len(hv))
                    mesh_vert.append(hv)
                    mesh_names.append(mname)
                    mesh_center.append(cen)
                geom_dataid[k] = mesh_names.index(mname)
                geom_pos[k] = geom_pos[k] + quat2mat(geom_quat[k]) @ mesh_center[geom_dataid[k]]
                geom_rbound[k] = np.linalg.norm(mesh_vert[geom_dataid[k]], axis=1).max()
            elif t == GEOM_BOX:
                geom_rbound[k] = np.linalg.norm(geom_size[k])
            elif t == GEOM_SPHERE:
                geom_rbound[k] = geom_size[k][0]
        # ---- sites
        ns = len(sites)
        site_bodyid = np.array([s["body"] for s in sites], np.int32)
        site_pos = np.array([_vec(s.get("pos", "0 0 0")) for s in sites]).reshape(ns, 3)
        site_quat = np.array([_quat_normalize(_vec(s.get("quat", "1 0 0 0"))) for s in sites]).reshape(ns, 4)
        # ---- actuators (general, joint transmission, gear[0] only)
        nu = len(self.actuators)
        actuator_trnid = np.zeros(nu, np.int32)
        actuator_gear = np.zeros(nu)
        actuator_gainprm = np.zeros((nu, 3))
        actuator_biasprm = np.zeros((nu, 3))
        actuator_ctrlrange = np.zeros((nu, 2))
        actuator_forcerange = np.zeros((nu, 2))
        actuator_ctrllimited = np.zeros(nu, np.int32)
        actuator_forcelimited = np.zeros(nu, np.int32)
        actuator_biastype = np.zeros(nu, np.int32)
        for i, a in enumerate(self.actuators):
            assert a["_tag"] == "general" and a.get("dyntype", "none") == "none"
            actuator_trnid[i] = jnames.index(a["joint"])
            actuator_gear[i] = _vec(a.get("gear", "1"))[0]
            actuator_gainprm[i] = _vec(a.get("gainprm", "1"), 3)[:3]
            actuator_biasprm[i] = _vec(a.get("biasprm", "0"), 3)[:3]
            actuator_biastype[i] = 1 if a.get("biastype", "none") == "affine" else 0
            if "ctrlrange" in a:
                actuator_ctrlrange[i] = _vec(a["ctrlrange"])
                actuator_ctrllimited[i] = 1 if self.c.autolimits or a.get("ctrllimited") == "true" else 0
            if "forcerange" in a:
                actuator_forcerange[i] = _vec(a["forcerange"])
                actuator_forcelimited[i] = 1 if self.c.autolimits or a.get("forcelimited") == "true" else 0
        # ---- equality (weld only)
        neq = len(self.eqs)
        eq_type = np.zeros(neq, np.int32)
        eq_obj1id = np.zeros(neq, np.int32)
        eq_obj2id = np.zeros(neq, np.int32)
        eq_solref = np.zeros((neq, 2))
        eq_solimp = np.zeros((neq, 5))
        eq_data = np.zeros((neq, 11))
        for i, e in enumerate(self.eqs):
            assert e["_tag"] == "weld"
            eq_type[i] = 1    # mjEQ_WELD
            eq_obj1id[i] = self.body_names.index(e["body1"])
            eq_obj2id[i] = self.body_names.index(e.get("body2", "world"))
            eq_solref[i] = _vec(e.get("solref", "0.02 1"))
            si = _vec(e.get("solimp", "0.9 0.95 0.001 0.5 2"))
            eq_solimp[i] = np.concatenate([si, _vec("0.9 0.95 0.001 0.5 2")[si.size:]])
            # anchor(3) relpos(3) relquat(4) torquescale(1); the env resets relpose to identity
            # (reference panda_env.py:329-335), so identity is stored directly.
            eq_data[i] = [0, 0, 0, 0, 0, 0, 1, 0, 0, 0, 1]

        opt = self.c.option
        out.update(dict(
            nq=nq, nv=nv, nu=nu, nbody=nb, njnt=nj, ngeom=ng, nsite=ns, nmocap=nmocap, neq=neq,
            nmesh=len(mesh_names),
            opt_timestep=opt["timestep"], opt_gravity=np.array(opt["gravity"], np.float64),
            opt_noslip_iterations=opt["noslip_iterations"], opt_iterations=opt["iterations"],
            opt_tolerance=opt["tolerance"], opt_multiccd=opt.get("multiccd", 0),
            opt_warmstart=opt.get("warmstart", 1), opt_cone_pyramidal=int(opt["cone"] == "pyramidal"),
            opt_integrator_euler=int(opt["integrator"] == "Euler"), opt_noslip_tolerance=opt["noslip_tolerance"],
            body_parentid=body_parentid, body_rootid=body_rootid, body_weldid=body_weldid,
            body_mocapid=body_mocapid, body_jntadr=body_jntadr, body_jntnum=body_jntnum,
            body_dofadr=body_dofadr, body_dofnum=body_dofnum, body_pos=body_pos, body_quat=body_quat,
            body_ipos=body_ipos, body_iquat=body_iquat, body_mass=body_mass, body_inertia=body_inertia,
            jnt_type=jnt_type, jnt_qposadr=jnt_qposadr, jnt_dofadr=jnt_dofadr, jnt_bodyid=jnt_bodyid,
            jnt_pos=jnt_pos, jnt_axis=jnt_axis, jnt_range=jnt_range, jnt_limited=jnt_limited,
            jnt_solref=jnt_solref, jnt_solimp=jnt_solimp, jnt_margin=jnt_margin,
            dof_armature=np.array(dof_armature), dof_damping=np.array(dof_damping),
            dof_jntid=np.array(dof_jntid, np.int32), dof_bodyid=np.array(dof_bodyid, np.int32),
            qpos0=np.array(qpos0, np.float64),
            geom_type=geom_type, geom_bodyid=geom_bodyid, geom_contype=geom_contype,
            geom_conaffinity=geom_conaffinity, geom_condim=geom_condim, geom_priority=geom_priority,
            geom_size=geom_size, geom_pos=geom_pos, geom_quat=geom_quat, geom_friction=geom_friction,
            geom_solref=geom_solref, geom_solimp=geom_solimp, geom_margin=geom_margin, geom_gap=geom_gap,
            geom_dataid=geom_dataid, geom_solmix=geom_solmix, geom_rbound=geom_rbound,
            mesh_vertadr=np.array(mesh_vertadr, np.int32), mesh_vertnum=np.array(mesh_vertnum, np.int32),
            mesh_vert=(np.concatenate(mesh_vert) if mesh_vert else np.zeros((0, 3))),
            site_bodyid=site_bodyid, site_pos=site_pos, site_quat=site_quat,
            actuator_trnid=actuator_trnid, actuator_gear=actuator_gear, actuator_gainprm=actuator_gainprm,
            actuator_biasprm=actuator_biasprm, actuator_biastype=actuator_biastype,
            actuator_ctrlrange=actuator_ctrlrange, actuator_forcerange=actuator_forcerange,
            actuator_ctrllimited=actuator_ctrllimited, actuator_forcelimited=actuator_forcelimited,
            eq_type=eq_type, eq_obj1id=eq_obj1id, eq_obj2id=eq_obj2id, eq_solref=eq_solref,
            eq_solimp=eq_solimp, eq_data=eq_data,
            names_body=np.array(self.body_names), names_jnt=np.array(jnames), names_geom=np.array(gnames),
            names_site=np.array(snames), names_mesh=np.array(mesh_names, dtype="U32"),
            names_actuator=np.array([a.get("name", "") for a in self.actuators]),
        ))
        from . import setconst
        out.update(setconst.compute(out))
        return out


DEFAULT_REFERENCE_XML = "/root/reference/panda_mujoco_gym/assets/shelf_pnp.xml"
DATA_PATH = os.path.join(os.path.dirname(__file__), "data", "panda_shelf.npz")


def compile_xml(xml_path=DEFAULT_REFERENCE_XML):
    return MJCFCompiler(xml_path).compile()


def main():
    import argparse
    ap = argparse.ArgumentParser(description="compile the shelf_pnp MJCF into panda_shelf.npz")
    ap.add_argument("--xml", default=DEFAULT_REFERENCE_XML)
    ap.add_argument("--out", default=DATA_PATH)
    args = ap.parse_args()
    m = compile_xml(args.xml)
    arrays = {k: np.asarray(v) for k, v in m.items()}
    if os.path.exists(args.out):
        old = np.load(args.out, allow_pickle=False)
        if set(old.files) == set(arrays) and all(np.array_equal(old[k], arrays[k]) for k in arrays):
            print(f"{args.out} up to date")
            return
    np.savez_compressed(args.out, **arrays)
    print(f"wrote {args.out}: nq={m['nq']} nv={m['nv']} nu={m['nu']} nbody={m['nbody']} "
          f"ngeom={m['ngeom']} nsite={m['nsite']} nmesh={m['nmesh']} hull verts={len(m['mesh_vert'])}")


if __name__ == "__main__":
    main()
