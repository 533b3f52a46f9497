"""CPU model of the fp32 Newton solve on the closed-finger (`pressed`) fixture's arm island: the
linear system of the oracle's final active set, H x = M x_smooth + J^T D aref, solved
  (a) in fp64 with fp64 data (reference), (b) in fp64 with the data rounded to fp32 (the data's
  own rounding), (c) by fp32 Cholesky with fp32 refinement steps (the round-4 kernel's second
  Newton iteration), (d) by fp32 Cholesky with refinement steps whose residual is accumulated in
  fp64 (the round-5 kernel, step.hip newton_refine_grad).
Prints each solution's error relative to |x| in the M-norm.  usage: python tools/mpir_model.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mujoco-panda-pnp_amd"), os.path.join(ROOT, "tests")]
import numpy as np
from oracle import oracle as O
from pnp_amd.model import load_model
import physics_states as PS, test_step_gpu as T
m=load_model(); nv=m.nv
pr = PS.reset_states(12, seed=11, model=m)
pr["qpos"][:, 7:9] = -np.linspace(0.001, 0.004, 12)[:, None]
pr["ctrl"][:, -2:] = 0.0
pr["qvel"] += np.random.default_rng(5).normal(size=pr["qvel"].shape) * 0.02
st=T._round32(pr)
f32=np.float32
def chol32(A):
    n=A.shape[0]; L=np.zeros_like(A,dtype=f32)
    A=A.astype(f32)
    for j in range(n):
        s=A[j,j]-np.dot(L[j,:j],L[j,:j]).astype(f32)
        L[j,j]=np.sqrt(f32(s))
        for i in range(j+1,n):
            L[i,j]=f32((A[i,j]-np.dot(L[i,:j],L[j,:j]).astype(f32))/L[j,j])
    return L
def solve32(L,b):
    b=b.astype(f32); n=len(b); y=np.zeros(n,f32)
    for i in range(n): y[i]=f32((b[i]-np.dot(L[i,:i],y[:i]).astype(f32))/L[i,i])
    x=np.zeros(n,f32)
    for i in reversed(range(n)): x[i]=f32((y[i]-np.dot(L[i+1:,i],x[i+1:]).astype(f32))/L[i,i])
    return x
sl=slice(0,9)
for b in range(12):
    f = O.forward_fields({k: st[k][b] for k in O.STATE_KEYS}, ["qM","efc_J","efc_D","efc_aref","efc_type","qacc_smooth","qacc_newton","nefc"], model=m)
    ne=int(f["nefc"][0]); M=f["qM"].reshape(nv,nv); J=f["efc_J"].reshape(ne,nv); D=f["efc_D"]; ar=f["efc_aref"]; xs=f["qacc_smooth"]; xn=f["qacc_newton"]
    act=(f["efc_type"]==0)|(J@xn-ar<0)
    Ja,Da,aa=J[act],D[act],ar[act]
    Ma=M[sl,sl]; Jt=Ja[:,sl]
    # arm island only (fingers + arm): other trees' columns ignored if rows touch only arm
    rows=np.abs(Ja[:,9:]).sum(1)==0
    Jt=Jt[rows]; Dt=Da[rows]; at=aa[rows]
    H=Ma+Jt.T@(Dt[:,None]*Jt); rhs=Ma@xs[sl]+Jt.T@(Dt*at)
    x64=np.linalg.solve(H,rhs)
    nrm=lambda v: np.sqrt(v@Ma@v)
    ref=nrm(x64)
    # data rounded to fp32, fp64 solve
    H2=Ma.astype(f32).astype(float)+Jt.astype(f32).astype(float).T@(Dt.astype(f32).astype(float)[:,None]*Jt.astype(f32).astype(float))
    rhs2=Ma.astype(f32).astype(float)@xs[sl].astype(f32).astype(float)+Jt.astype(f32).astype(float).T@(Dt.astype(f32)*at.astype(f32)).astype(float)
    xd=np.linalg.solve(H2,rhs2)
    # fp32 everything
    H32=(Ma.astype(f32)+Jt.astype(f32).T@(Dt.astype(f32)[:,None]*Jt.astype(f32))).astype(f32)
    L=chol32(H32)
    def grad32(x):  # fp32 gradient g = M(x-xs) + J^T D (J x - a)
        x=x.astype(f32); jar=(Jt.astype(f32)@x - at.astype(f32)).astype(f32)
        return (Ma.astype(f32)@(x-xs[sl].astype(f32)) + Jt.astype(f32).T@(Dt.astype(f32)*jar)).astype(f32)
    def grad64(x):
        x=x.astype(f32).astype(float); J32=Jt.astype(f32).astype(float); jar=J32@x - at.astype(f32).astype(float)
        return Ma.astype(f32).astype(float)@(x-xs[sl].astype(f32).astype(float)) + J32.T@(Dt.astype(f32).astype(float)*jar)
    x0=np.zeros(9,f32)
    x1=(x0-solve32(L,grad32(x0))).astype(f32)
    x2=(x1-solve32(L,grad32(x1))).astype(f32)
    x3=(x2-solve32(L,grad32(x2))).astype(f32)
    y2=(x1-solve32(L,grad64(x1).astype(f32))).astype(f32)
    y3=(y2-solve32(L,grad64(y2).astype(f32))).astype(f32)
    ev=np.linalg.eigvalsh(H); 
    print(f"env {b} rows {rows.sum()} cond(H) {ev.max()/ev.min():.2e}: data-rounding {nrm(xd-x64)/ref:.2e}; fp32 1 step {nrm(x1-x64)/ref:.2e}, +1 refine {nrm(x2-x64)/ref:.2e}, +2 {nrm(x3-x64)/ref:.2e}; fp64-residual refine {nrm(y2-x64)/ref:.2e}, +2 {nrm(y3-x64)/ref:.2e}")
