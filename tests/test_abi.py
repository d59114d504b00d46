"""The C-ABI library loads and exports every entry point include/*.h
declares (no GPU calls), and the gfx950 code keeps the parity-critical
arithmetic free of FMA contraction."""
from __future__ import annotations

import os
import re
import subprocess

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "distlr_amd.h")
LIB = os.path.join(ROOT, "dist-lr_amd", "lib", "libdistlr_amd.so")


def declared_functions():
    with open(HEADER) as f:
        text = f.read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(dlr_[a-z0-9_]+)\s*\(", text)))


def exported_symbols():
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], check=True, capture_output=True, text=True).stdout
    return {line.split()[-1] for line in out.splitlines() if line.strip()}


def test_header_declares_entry_points():
    funcs = declared_functions()
    assert len(funcs) >= 25
    assert "dlr_train_step" in funcs and "dlr_create" in funcs


def test_library_exports_every_declared_symbol():
    missing = [f for f in declared_functions() if f not in exported_symbols()]
    assert not missing, missing


def test_python_binding_covers_header():
    import distlr_amd
    assert sorted(distlr_amd.SYMBOLS) == declared_functions()


def test_tuning_struct_matches_header_and_env(monkeypatch):
    # dlr_tuning: the binding's fields are the header's, in order; every
    # field AUTO by default; dlr_tuning_from_env parses the environment as
    # the engine reads it (no GPU needed)
    import distlr_amd
    with open(os.path.join(ROOT, "include", "distlr_amd.h")) as f:
        h = f.read()
    body = re.search(r"typedef struct dlr_tuning \{(.*?)\} dlr_tuning;", h, re.S).group(1)
    fields = re.findall(r"(\w+)(?=[,;])", re.sub(r"int64_t", "", body))
    assert [n for n, _ in distlr_amd.Tuning._fields_] == fields
    assert all(v == distlr_amd.AUTO for v in distlr_amd.Tuning.default().as_dict().values())
    for k in [k for k in os.environ if k.startswith("DLR_")]:
        monkeypatch.delenv(k)
    monkeypatch.setenv("DLR_GRAD_KERNEL", "touched")
    monkeypatch.setenv("DLR_PM", "1")
    monkeypatch.setenv("DLR_PM_MG", "0")
    monkeypatch.setenv("DLR_BAND_ROWS", "8192")
    monkeypatch.setenv("DLR_DENSE_GRAD", "blocked")
    t = distlr_amd.Tuning.from_env().as_dict()
    assert t["grad_layout"] == distlr_amd.LAYOUT_TOUCHED and t["product_margin"] == 1
    assert t["pm_in_gradient"] == 0 and t["band_rows"] == 8192 and t["dense_grad"] == 1
    assert t["pm_fused"] == distlr_amd.AUTO and t["hot_stream"] == distlr_amd.AUTO


def test_library_links_hip_and_rccl():
    out = subprocess.run(["readelf", "-d", LIB], check=True, capture_output=True, text=True).stdout
    assert "libamdhip64" in out and "librccl" in out


def test_library_has_gfx950_code_object():
    # The fat binary embeds an offload bundle whose target id names the arch.
    with open(LIB, "rb") as f:
        blob = f.read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob


def _kernel_bodies(asm: str):
    bodies, cur, name = {}, [], None
    for line in asm.splitlines():
        m = re.match(r"^(_Z\S+):", line)
        if m:
            name, cur = m.group(1), []
            continue
        if name:
            if "s_endpgm" in line:
                bodies[name] = cur
                name = None
            else:
                cur.append(line.strip())
    return bodies


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc"), reason="hipcc not available")
def test_no_fma_contraction_in_parity_kernels():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "dist-lr_amd"), "asm"], check=True)
    with open(os.path.join(ROOT, "dist-lr_amd", "build", "dlr_kernels.s")) as f:
        bodies = _kernel_bodies(f.read())
    assert bodies
    for name, body in bodies.items():
        ops = [l.split()[0] for l in body if l and not l.startswith((";", "."))]
        fma = sum(op in ("v_fma_f32", "v_fmac_f32_e32", "v_fmac_f32_e64", "v_pk_fma_f32", "v_mad_f32")
                  for op in ops)
        fixups = sum(op == "v_div_fixup_f32" for op in ops)
        # Only correctly-rounded f32 divisions (div_scale .. div_fixup: 3 fma +
        # 2 fmac each) may use fused f32 ops; sums and products must not.
        assert fma == 5 * fixups, (name, fma, fixups)
        if "margin" in name or "predict" in name:
            assert fma == 0, name


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc"), reason="hipcc not available")
def test_hand_placed_vmcnt_waits_cover_the_lds_dma():
    # The LDS-DMA residual fills of k_grad_lds are not tracked by the
    # compiler; the kernel waits for them with hand-placed s_waitcnt vmcnt.
    # A wait vmcnt(N) with N > 0 (loads issued after the fill stay in
    # flight) covers the fill only if at least N vector-memory instructions
    # issue between the fill's last global_load_lds and the wait, or the
    # compiler drained the counter (vmcnt(0)) in between.  The
    # current kernel waits vmcnt(0); this keeps any future partial wait
    # honest.  Checked on the gfx950 code of every instantiation.
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "dist-lr_amd"), "asm"], check=True)
    with open(os.path.join(ROOT, "dist-lr_amd", "build", "dlr_kernels.s")) as f:
        bodies = _kernel_bodies(f.read())
    grads = {n: b for n, b in bodies.items() if "k_grad_lds" in n}
    assert len(grads) >= 16, sorted(bodies)
    vmem = re.compile(r"^(global|buffer|flat)_(load|store|atomic)")
    for name, body in grads.items():
        asm_block = False
        for k, l in enumerate(body):
            if l.startswith(";;#ASMSTART"):
                asm_block = True
                continue
            if l.startswith(";;#ASMEND"):
                asm_block = False
                continue
            m = re.match(r"s_waitcnt vmcnt\((\d+)\)$", l)
            if not (asm_block and m and int(m.group(1)) > 0):
                continue
            want = int(m.group(1))
            fills = [q for q in range(k) if body[q].startswith("global_load_lds")]
            if not fills:
                continue
            between = body[fills[-1] + 1:k]
            # The N youngest operations at the wait must all come after the
            # fill: either on one straight path from the fill to the wait
            # (no label: no other path joins it; branches out of it do not
            # reach the wait), or -- the double-buffered form, whose group
            # loop lies between -- issued on the straight run that leaves the
            # fill, before its first label, which every path to the wait
            # passes (and no path back to the fill: the fill is the last
            # before the wait).
            joins = [q for q, x in enumerate(between) if x.startswith(".LBB")]
            run = between[:joins[0]] if joins else between
            drained = any(re.match(r"s_waitcnt vmcnt\(0\)", x) for x in run)
            issued = sum(bool(vmem.match(x)) for x in run)
            assert drained or issued >= want, (name, issued, want, "joins" if joins else "straight")
