"""CPU-side checks (no GPU): the C-ABI library loads and exports every symbol
include/mdl_engine.h declares, the ctypes struct matches the C layout, the
host-built rank tables order the reference's fp64 sort keys, and the host
packing / action encoding logic."""
import ctypes as C
import os
import re
import subprocess
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "mdl_engine.h")


_REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_symbols():
    txt = open(HEADER).read()
    return re.findall(r"^(?:int|const char\*)\s+(mdl_\w+)\(", txt, re.M)


def test_library_exports_every_header_symbol():
    from marl_gpu import _lib
    L = _lib.lib()
    syms = _header_symbols()
    assert len(syms) >= 14
    for s in syms:
        assert hasattr(L, s), s
        assert s in _lib.SIGNATURES, f"{s} missing a ctypes signature"
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    for s in syms:
        assert re.search(rf"\bT {s}\b", out), f"{s} not exported"
    assert L.mdl_version().startswith(b"mdl-engine")


def test_library_has_gfx950_code_object():
    from marl_gpu import _lib
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"hipv4-amdgcn-amd-amdhsa--gfx950" in blob or b"amdgcn-amd-amdhsa--gfx950" in blob


def test_makefile_lists_every_kernel_header():
    """Every header under csrc/ and include/ is a dependency of the library's objects in the Makefile
    (a header missing from HDR left a stale kernel in libmdl.so after an edit, round 6)."""
    mk = open(os.path.join(REPO, "marl-delivery_amd", "Makefile")).read()
    hdr = re.search(r"^HDR\s*=\s*(.*)$", mk, re.M).group(1).split()
    for f in sorted(os.listdir(os.path.join(REPO, "marl-delivery_amd", "csrc"))):
        if f.endswith(".hpp"):
            assert "csrc/" + f in hdr, f"csrc/{f} missing from the Makefile's HDR"
    assert "../include/mdl_engine.h" in hdr


def test_header_constants_match_python_binding():
    """Every integer #define MDL_* of include/mdl_engine.h that the ctypes binding names (tracker modes,
    action formats, builders, step layouts incl. HALVES, limits, reward-term bits) has the same value."""
    from marl_gpu import _lib
    txt = open(os.path.join(REPO, "include", "mdl_engine.h")).read()
    defs = {m.group(1): int(m.group(2)) for m in re.finditer(r"^#define (MDL_[A-Z0-9_]+)\s+(\d+)\b", txt, re.M)}
    named = [k for k in defs if hasattr(_lib, k)]
    assert {"MDL_STEP_LAYOUT_AUTO", "MDL_STEP_LAYOUT_WAVE", "MDL_STEP_LAYOUT_ROWS", "MDL_STEP_LAYOUT_HALVES",
            "MDL_TRACKER_MAPPO_STALE", "MDL_ACTION_CODES", "MDL_OBS_BUILDER_GENERIC"} <= set(named)
    for k in named:
        assert getattr(_lib, k) == defs[k], k
    from marl_gpu import engine
    assert set(engine.STEP_LAYOUTS.values()) == {defs[k] for k in defs if k.startswith("MDL_STEP_LAYOUT_")}


def test_config_struct_layout_matches_c(tmp_path):
    from marl_gpu import _lib
    src = tmp_path / "probe.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "mdl_engine.h"\n'
                   'int main(){printf("%zu %zu %zu %zu\\n", sizeof(MdlConfig), offsetof(MdlConfig, shaping),'
                   ' offsetof(MdlConfig, obs_max_time_steps), offsetof(MdlConfig, max_packages_state));return 0;}\n')
    exe = tmp_path / "probe"
    subprocess.check_call(["gcc", "-I", os.path.join(REPO, "include"), str(src), "-o", str(exe)])
    got = [int(x) for x in subprocess.check_output([str(exe)]).split()]
    M = _lib.MdlConfig
    assert got == [C.sizeof(M), M.shaping.offset, M.obs_max_time_steps.offset, M.max_packages_state.offset]


def _py_key(dr, dc, H, W):
    return (dr / H) ** 2 + (dc / W) ** 2     # MAPPO/helper.py:139 key, CPython float arithmetic


@pytest.mark.parametrize("H,W", [(10, 10), (20, 20), (7, 7), (41, 41), (64, 64), (5, 13), (1, 3)])
def test_rank_table_orders_python_fp64_keys(H, W):
    from marl_gpu import _lib
    n = (2 * H - 1) * (2 * W - 1)
    out = np.zeros(n, np.uint16)
    assert _lib.lib().mdl_rank_table(H, W, out.ctypes.data) == 0
    keys = np.array([_py_key(dr, dc, H, W) for dr in range(-(H - 1), H) for dc in range(-(W - 1), W)])
    u = np.unique(keys)
    want = np.searchsorted(u, keys)
    np.testing.assert_array_equal(out, want)


def test_rank_table_differs_from_integer_distance():
    """SURVEY hard part 3: the fp64 key order is not the integer dr^2+dc^2 order."""
    from marl_gpu import _lib
    H = W = 10
    out = np.zeros((2 * H - 1) * (2 * W - 1), np.uint16)
    _lib.lib().mdl_rank_table(H, W, out.ctypes.data)
    # equal integer distances may map to distinct fp64 keys (and vice versa): just check both orders agree on
    # strict integer inequalities where the fp64 keys agree too
    idx = [(dr, dc) for dr in range(-(H - 1), H) for dc in range(-(W - 1), W)]
    ints = np.array([dr * dr + dc * dc for dr, dc in idx])
    ties_int = sum(1 for i in range(0, len(idx), 7) for j in range(0, len(idx), 5)
                   if ints[i] == ints[j] and out[i] != out[j])
    assert ties_int > 0


def test_encode_actions_and_pack_view():
    from marl_gpu.compat import encode_actions
    from marl_gpu.helper import pack_view
    codes = encode_actions([("S", "0"), ("L", "1"), ("R", "2"), ("U", "3"), ("D", "x"), ("Q", "1")], 6)
    assert codes.tolist() == [0, 1 | 8, 2 | 16, 3 | 24, 4 | 24, 5 | 8]
    with pytest.raises(ValueError):
        encode_actions([("S", "0")], 2)
    rec = pack_view(7, [(2, 3, 0), (5, 5, 4)], [[4, 1, 1, 1, 2, 2, 3, 30]], 10, 10)
    assert rec.tolist()[:4] == [7, 2, 1, 0]
    assert rec.tolist()[4:10] == [1, 2, 0, 4, 4, 4]
    with pytest.raises(ValueError):
        pack_view(0, [(11, 1, 0)], [], 10, 10)


def test_trainer_int_decode_matches_labelencoder():
    """MAPPO/trainer.py:84-89,198-205: LabelEncoder sorts classes -> D,L,R,S,U."""
    from sklearn.preprocessing import LabelEncoder
    le = LabelEncoder().fit(["S", "L", "R", "U", "D"])
    assert list(le.classes_) == ["D", "L", "R", "S", "U"]
    from golden_io import TRAINER_MOVE_CODES
    from marl_gpu.compat import MOVE_CODES
    assert [MOVE_CODES[m] for m in le.classes_] == TRAINER_MOVE_CODES.tolist()


def test_builtin_maps_load_like_reference():
    from marl_gpu.maps import BUILTIN, load_map, map_path
    for m in BUILTIN:
        g = np.asarray(load_map(map_path(m)))
        assert g.ndim == 2 and set(np.unique(g)) <= {0, 1}
    assert np.asarray(load_map(map_path("map1"))).shape == (10, 10)
    assert np.asarray(load_map(map_path("synthetic64"))).shape == (64, 64)


def test_product_has_no_oracle_dependency():
    """The product package never imports the CPU oracle (test infrastructure)."""
    pkg = os.path.join(REPO, "marl-delivery_amd", "marl_gpu")
    for root, _, files in os.walk(pkg):
        for f in files:
            if f.endswith(".py"):
                txt = open(os.path.join(root, f)).read()
                assert "import oracle" not in txt and "from oracle" not in txt, f
    for f in os.listdir(os.path.join(REPO, "marl-delivery_amd", "csrc")):
        txt = open(os.path.join(REPO, "marl-delivery_amd", "csrc", f)).read()
        assert "mdl_oracle" not in txt and "liboracle" not in txt, f
    mk = open(os.path.join(REPO, "marl-delivery_amd", "Makefile")).read()
    assert "oracle" not in mk


def _bench_module():
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_under_test", os.path.join(_REPO, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_bench_gpus_n_self_launches_torchrun_without_touching_the_gpu(monkeypatch):
    """`python bench.py --gpus 8 ...` outside torchrun: the parent starts
    `python -m torch.distributed.run --nproc-per-node 8 bench.py <same args>` as a child and
    returns its exit code, and makes no GPU call of its own (a GPU-initialising parent must not
    spawn or exec GPU children on this pool)."""
    import torch
    bench = _bench_module()
    monkeypatch.delenv("WORLD_SIZE", raising=False)

    def no_gpu(*a, **k):
        raise AssertionError("the launching parent touched the GPU")
    for name in ("is_available", "init", "set_device", "synchronize", "current_device", "device_count"):
        monkeypatch.setattr(torch.cuda, name, no_gpu)
    seen = {}

    def fake_forward(cmd, env=None):
        seen["cmd"], seen["env"] = cmd, env
        return 7
    monkeypatch.setattr(bench, "forward_child", fake_forward)
    argv = ["--gpus", "8", "--steps", "20", "--warmup", "5"]
    assert bench.main(argv) == 7
    cmd = seen["cmd"]
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-len(argv) - 1] == os.path.join(_REPO, "bench.py") and cmd[-len(argv):] == argv
    assert seen["env"]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0" and seen["env"]["MDL_BENCH_LAUNCHER"] == "self"


def test_bench_forward_child_passes_only_the_json_line(capfd):
    """The self-launching parent forwards rank 0's JSON line to stdout, every other line of the
    child to stderr, and the child's exit code."""
    bench = _bench_module()
    code = ("import json, sys; print('torchrun chatter'); print(json.dumps({'metric': 'm', 'value': 1})); "
            "sys.stdout.flush(); sys.exit(3)")
    assert bench.forward_child([sys.executable, "-c", code]) == 3
    out, err = capfd.readouterr()
    assert out.strip() == '{"metric": "m", "value": 1}' and "torchrun chatter" in err


def test_bench_rank_count_must_match_gpus():
    """Under torchrun (WORLD_SIZE set) --gpus must equal the rank count."""
    env = dict(os.environ, WORLD_SIZE="1")
    out = subprocess.run([sys.executable, os.path.join(_REPO, "bench.py"), "--gpus", "2", "--steps", "5"], cwd=_REPO,
                         capture_output=True, text=True, timeout=120, env=env)
    assert out.returncode != 0 and "WORLD_SIZE=1" in out.stderr


LLVM_BIN = "/opt/rocm/lib/llvm/bin"


def _kernel_resources(so_path, tmp_path):
    """Per-kernel (private segment bytes, SGPRs, VGPRs) of every gfx950 code object in the
    library's .hip_fatbin (clang offload bundles, one per translation unit), from the code
    objects' AMDGPU metadata notes."""
    import struct
    fat = tmp_path / "fat.bin"
    subprocess.check_call([f"{LLVM_BIN}/llvm-objcopy", "--dump-section", f".hip_fatbin={fat}", so_path,
                           str(tmp_path / "dummy.so")])
    b = fat.read_bytes()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    res = {}
    for k, m in enumerate(re.finditer(re.escape(magic), b)):
        s = m.start()
        n, = struct.unpack_from("<Q", b, s + 24)
        off = s + 32
        for _ in range(n):
            o, sz, tl = struct.unpack_from("<QQQ", b, off)
            triple = b[off + 24:off + 24 + tl].decode()
            off += 24 + tl
            if "gfx950" not in triple or sz == 0:
                continue
            co = tmp_path / f"k{k}.co"
            co.write_bytes(b[s + o:s + o + sz])
            notes = subprocess.run([f"{LLVM_BIN}/llvm-readelf", "--notes", str(co)], capture_output=True,
                                   text=True, check=True).stdout
            name = None
            for line in notes.splitlines():   # keys after .name, alphabetically: .private.., .sgpr.., .vgpr..
                t = line.split()
                if len(t) == 2 and t[0] == ".name:":
                    name = t[1]
                    res[name] = {}
                elif name and len(t) == 2 and t[0] in (".private_segment_fixed_size:", ".sgpr_count:", ".sgpr_spill_count:",
                                                               ".vgpr_count:"):
                    res[name][t[0][1:-1]] = int(t[1])
    return res


@pytest.mark.skipif(not os.path.exists(f"{LLVM_BIN}/llvm-readelf"), reason="ROCm LLVM tools absent")
def test_step_kernels_fit_eight_waves_without_scratch(tmp_path):
    """The per-launch step kernels of one and two package chunks (P <= 128: configs 1-5) and the
    fused step + observation kernel are compiled for 8 waves per SIMD (amdgpu_waves_per_eu(8),
    csrc/mdl_kernels.hip step_wpe): their registers fit the 8-wave budget (<= 64 VGPRs,
    <= 96 SGPRs) with no spill to scratch.  Config 5 ran 12 % slower at the compiler's own 7."""
    from marl_gpu import _lib
    res = _kernel_resources(_lib.LIB_PATH, tmp_path)
    step = [n for n in res if re.search(r"k_stepILb[01]ELi[12]ELb0ELi\d+EE", n) or "k_step_obs" in n]
    assert len(step) >= 20, step   # 2 tracker modes x 2 chunkings x 4 robot specialisations + step_obs
    for n in step:
        r = res[n]
        assert r["private_segment_fixed_size"] == 0, (n, r)
        assert r["vgpr_count"] <= 64 and r["sgpr_count"] <= 96, (n, r)
    # the headline kernel and config 5's are among them
    assert any("k_stepILb1ELi1ELb0ELi5EE" in n for n in step) and any("k_stepILb1ELi2ELb0ELi16EE" in n for n in step)
    # no hot-path kernel spills: scratch only where a wide variant needs it
    spill = sorted(n for n, r in res.items() if r.get("private_segment_fixed_size", 0) > 0
                   and re.search(r"k_step|k_obs|k_reset|k_seed", n))
    assert not spill, spill


@pytest.mark.skipif(not os.path.exists(f"{LLVM_BIN}/llvm-readelf"), reason="ROCm LLVM tools absent")
def test_rows_step_kernels_have_no_scratch(tmp_path):
    """k_step_rows (four envs per wavefront, csrc/mdl_step_rows.hpp): one instantiation per tracker mode,
    robot specialisation (A == 5, A <= 8) and full-chunk count (NFULL 0 or 3), four package chunks; no
    spill to scratch; config 4's form (stale tracker, A == 5, NFULL 3) within 72 VGPRs (7 waves per
    SIMD, the occupancy profiles/r06/ab10 was measured at), the other A == 5 forms within 104, the
    A <= 8 forms within 128 (4 waves); no SGPR spill in the A == 5 forms."""
    from marl_gpu import _lib
    res = _kernel_resources(_lib.LIB_PATH, tmp_path)
    rows = [n for n in res if "k_step_rows" in n]
    assert len(rows) == 8, rows
    for n in rows:
        assert res[n]["private_segment_fixed_size"] == 0, (n, res[n])
        cap = 72 if "k_step_rowsILb1ELi5ELi4ELi3E" in n else 104 if "ILi5ELi4E" in n else 128
        assert res[n]["vgpr_count"] <= cap, (n, res[n])
        if "ILi5ELi4E" in n:   # the A == 5 forms (configs 4 and 2 at >= 7,168 envs): no SGPR spill
            assert res[n].get("sgpr_spill_count", 0) == 0, (n, res[n])


@pytest.mark.skipif(not os.path.exists(f"{LLVM_BIN}/llvm-readelf"), reason="ROCm LLVM tools absent")
def test_halves_step_kernels_have_no_scratch(tmp_path):
    """k_step_halves (two envs per wavefront, csrc/mdl_step_halves.hpp): one instantiation per tracker
    mode and full-chunk count (NFULL 0 or 3); no spill to scratch or SGPR spill; config 5's form (stale
    tracker, NFULL 3) within 72 VGPRs (7 waves per SIMD, profiles/r06/ab9), the others within 80."""
    from marl_gpu import _lib
    res = _kernel_resources(_lib.LIB_PATH, tmp_path)
    halves = [n for n in res if "k_step_halves" in n]
    assert len(halves) == 4, halves
    for n in halves:
        assert res[n]["private_segment_fixed_size"] == 0, (n, res[n])
        assert res[n].get("sgpr_spill_count", 0) == 0, (n, res[n])
        assert res[n]["vgpr_count"] <= (72 if "k_step_halvesILb1ELi3E" in n else 80), (n, res[n])


def test_bench_step_layout_flag():
    """bench.py --step-layout reaches BatchedEnv (MdlConfig.step_layout); auto is the default."""
    bench = _bench_module()
    assert bench.parse([]).step_layout == "auto"
    assert bench.parse(["--config", "4", "--step-layout", "wave"]).step_layout == "wave"
    with pytest.raises(SystemExit):
        bench.parse(["--step-layout", "diagonal"])


_PROFILING_SWITCHES = ["MDL_EXP_NOWAIT", "MDL_EXP_NOTUPLES", "MDL_EXP_NOLDS", "MDL_ABLATE=1", "MDL_STAMPS"]


@pytest.mark.parametrize("switch", _PROFILING_SWITCHES)
def test_profiling_switches_need_a_profiling_build(switch):
    """A switch that changes what the kernels compute is an #error unless the build says it is a
    profiling build; with -DMDL_PROFILING_BUILD it preprocesses."""
    pkg = os.path.join(REPO, "marl-delivery_amd")
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "--cuda-device-only", "-std=c++17", "-E",
           "-I", os.path.join(REPO, "include"), "-I", os.path.join(pkg, "csrc"),
           os.path.join(pkg, "csrc", "mdl_kernels.hip"), "-o", os.devnull]
    bad = subprocess.run(cmd + ["-D" + switch], capture_output=True, text=True)
    assert bad.returncode != 0 and "MDL_PROFILING_BUILD" in bad.stderr, bad.stderr[-500:]
    ok = subprocess.run(cmd + ["-D" + switch, "-DMDL_PROFILING_BUILD"], capture_output=True, text=True)
    assert ok.returncode == 0, ok.stderr[-500:]


def test_product_library_has_no_profiling_code():
    """The shipped libmdl.so carries no diagnostic stamp buffer (MDL_STAMPS builds define g_stamps)."""
    from marl_gpu import _lib
    assert b"g_stamps" not in open(_lib.LIB_PATH, "rb").read()


def test_lib_path_override_needs_profiling_flag():
    """MDL_LIB_PATH selects a profiling build; without MDL_PROFILING=1 the import refuses it
    instead of loading another library."""
    env = dict(os.environ, MDL_LIB_PATH="/nonexistent/libmdl.so")
    env.pop("MDL_PROFILING", None)
    env["PYTHONPATH"] = os.path.join(REPO, "marl-delivery_amd")
    r = subprocess.run([sys.executable, "-c", "import marl_gpu._lib"], env=env, capture_output=True, text=True)
    assert r.returncode != 0 and "MDL_PROFILING=1" in r.stderr, r.stderr[-500:]


def test_traffic_json_recomputes_from_committed_profiles(tmp_path):
    """bench.py's roofline.traffic comes from profiles/traffic.json; every record in it is recomputed
    here from the per-dispatch PMC rows committed under profiles/ and the committed FETCH_SIZE
    calibration (the measurement record is self-contained)."""
    import json
    tj = json.load(open(os.path.join(REPO, "profiles", "traffic.json")))
    specs = []
    for rec in tj["records"]:
        src = rec["source"].split(" ", 1)[0]
        assert src.startswith("profiles/") and os.path.isdir(os.path.join(REPO, src)), src
        c = rec["config"]
        specs.append(f"{rec['name']}={os.path.join(REPO, src)}:{c['envs']},{c['agents']},{c['packages']},"
                     + "+".join(c["maps"]) + f":{rec['kernel'].replace('mdl::', '')}:{int(bool(rec.get('obs')))}")
    out = tmp_path / "traffic.json"
    subprocess.check_call([sys.executable, os.path.join(REPO, "scripts", "traffic_json.py"), str(out),
                           os.path.join(REPO, tj["calibration"])] + specs, stdout=subprocess.DEVNULL)
    again = json.load(open(out))
    for a, b in zip(tj["records"], again["records"]):
        assert a["hbm_bytes_per_launch"] == b["hbm_bytes_per_launch"], a["name"]
        assert a["fetch_dispatches"] == b["fetch_dispatches"] >= 100


def test_product_sources_have_no_variant_switches():
    """the product kernels carry no compile-time A/B switches (the non-default
    branches of round 4's experiments are deleted; the history keeps them) and read no environment
    overrides.  The only preprocessor switches left are the profiling-only ones, each an #error
    without -DMDL_PROFILING_BUILD (test_profiling_switches_need_a_profiling_build)."""
    fenced = {"MDL_EXP_NOWAIT", "MDL_EXP_NOTUPLES", "MDL_EXP_NOLDS", "MDL_ABLATE", "MDL_STAMPS", "MDL_PROFILING_BUILD"}
    srcs = [os.path.join(REPO, "marl-delivery_amd", "csrc", f) for f in os.listdir(os.path.join(REPO, "marl-delivery_amd", "csrc"))]
    srcs.append(os.path.join(REPO, "include", "mdl_engine.h"))
    seen = set()
    for path in srcs:
        txt = open(path).read()
        assert "getenv" not in txt, path
        for m in re.finditer(r"^\s*#\s*(?:if|ifdef|ifndef|elif)\b(.*)$", txt, re.M):
            for name in re.findall(r"\b(MDL_[A-Z0-9_]+)", m.group(1)):
                seen.add(name)
                assert name in fenced or name == "MDL_ENGINE_H", (path, m.group(0))
    assert {"MDL_ABLATE", "MDL_STAMPS"} <= seen
