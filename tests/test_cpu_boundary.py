"""The C-ABI library loads on a GPU-less host and exports exactly what include/tt_mi355x.h declares;
argument validation errors come back as status codes with a message (no compute is launched)."""
import re
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


def _declared():
    text = (ROOT / "include" / "tt_mi355x.h").read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(tt_[a-z0-9_]+)\s*\(", text)))


@pytest.fixture(scope="module")
def lib():
    from two_tower_recommender_model_amd import _lib
    from two_tower_recommender_model_amd.build import LIB, build

    build()
    return _lib.load()


def test_every_declared_symbol_exported(lib):
    from two_tower_recommender_model_amd import _lib
    from two_tower_recommender_model_amd.build import LIB

    out = subprocess.run(["nm", "-D", "--defined-only", str(LIB)], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (tt_[a-z0-9_]+)", out))
    declared = _declared()
    assert declared, "header parse failed"
    missing = [d for d in declared if d not in exported]
    assert not missing, missing
    extra = sorted(exported - set(declared))
    assert not extra, f"exported but not declared in the header: {extra}"
    assert sorted(_lib.SIGNATURES) == declared
    assert lib.tt_num_entry_points() == len(_lib.COMPUTE_ENTRY_POINTS)
    assert lib.tt_abi_version() == 4


def test_launch_plan_layout_matches_the_header(tmp_path):
    """The ctypes mirror of tt_launch_plan_t (and its role structs) has the C compiler's layout:
    sizes and field offsets from a C program built against include/tt_mi355x.h."""
    import ctypes as C

    from two_tower_recommender_model_amd import _lib

    structs = {"tt_launch_plan_t": _lib.LaunchPlan, "tt_wgrad_role_t": _lib.WgradRole,
               "tt_update_role_t": _lib.UpdateRole, "tt_insert_role_t": _lib.InsertRole,
               "tt_resolve_role_t": _lib.ResolveRole, "tt_adagrad_role_t": _lib.AdagradRole,
               "tt_route_role_t": _lib.RouteRole, "tt_gather_role_t": _lib.GatherRole, "tt_peer_put_t": _lib.PeerPut,
               "tt_peer_direct_t": _lib.PeerDirect, "tt_peer_wait_t": _lib.PeerWait}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "tt_mi355x.h"', "int main(void) {"]
    for cname, py in structs.items():
        lines.append(f'  printf("{cname} sizeof %zu\\n", sizeof({cname}));')
        for fname, _ in py._fields_:
            lines.append(f'  printf("{cname} {fname} %zu\\n", offsetof({cname}, {fname}));')
    lines.append("  return 0;\n}")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c11", f"-I{ROOT / 'include'}", str(src), "-o", str(exe)], check=True)
    got = {}
    for line in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.splitlines():
        cname, fname, v = line.split()
        got[(cname, fname)] = int(v)
    for cname, py in structs.items():
        assert got[(cname, "sizeof")] == C.sizeof(py), cname
        for fname, _ in py._fields_:
            assert got[(cname, fname)] == getattr(py, fname).offset, (cname, fname)


def test_launch_rejects_unknown_role_sets(lib):
    """tt_launch runs only the fused launches the library implements; another role set, or a role
    flag that contradicts the launch, is a status code, not a launch."""
    import ctypes as C

    from two_tower_recommender_model_amd import _lib

    plan = _lib.LaunchPlan(roles=_lib.ROLE_GATHER | _lib.ROLE_WGRAD)
    assert lib.tt_launch(C.byref(plan), None) == 1001
    assert b"set of roles" in lib.tt_last_error_string()
    plan = _lib.LaunchPlan(roles=_lib.ROLE_WGRAD | _lib.ROLE_INSERT | _lib.ROLE_ADAGRAD)  # ring tail: multi_only
    assert lib.tt_launch(C.byref(plan), None) == 1001
    assert b"multi_only" in lib.tt_last_error_string()
    plan = _lib.LaunchPlan(roles=_lib.ROLE_WGRAD | _lib.ROLE_INSERT | _lib.ROLE_ADAGRAD, B=8192,
                           adagrad=_lib.AdagradRole(multi_only=1, B=4096))
    assert lib.tt_launch(C.byref(plan), None) == 1001
    assert b"adagrad.B" in lib.tt_last_error_string()
    assert lib.tt_launch(None, None) == 1001


def test_errors_are_status_codes(lib):
    rc = lib.tt_pooled_fwd(None, None, 0, None, 0, 0, None, 0, None, 0, None, 0, 0, None, None)
    assert rc == 1001
    assert b"table count" in lib.tt_last_error_string()
    rc = lib.tt_linear_fwd(3, None, 2, 0, None, None, 1, 1, 1, None, 0, 1, 3, None)
    assert rc == 1001 and b"groups" in lib.tt_last_error_string()


def test_workspace_queries(lib):
    assert lib.tt_bwd_workspace_bytes(16384) > 16384 * 4 * 5
    assert lib.tt_linear_bwd_weight_workspace_bytes(2, 8192, 128, 128) > 0
    assert lib.tt_dot_bce_workspace_bytes(8192) >= 8192 * 4


def test_product_path_has_no_cpu_fallback():
    import torch

    from two_tower_recommender_model_amd import _lib, ops

    with pytest.raises(_lib.TTError):
        ops.complete_cumsum(torch.zeros(4, dtype=torch.int32))
    src = "\n".join(p.read_text() for p in (ROOT / "two_tower_recommender_model_amd").rglob("*.py"))
    assert "import oracle" not in src and "from oracle" not in src


def test_tower_shape_flags_validated(lib):
    """tt_tower_shape_t.flags (ABI 2; `_pad` in ABI 1): unknown bits are TT_EINVAL, and a
    TT_TOWER_GENERAL_T1 shape is refused by every T1 entry point except the indexed multi-feature
    one (its strips are tile-major; the row-owned T1 and tower_l2_kernel write row-major ones)."""
    import ctypes as C

    from two_tower_recommender_model_amd import _lib

    def shape(flags):
        return _lib.TowerShape(L=2, width=(C.c_int32 * 4)(128, 64, 0, 0), in_dim=(C.c_int32 * 2)(128, 128),
                               in_col=(C.c_int32 * 2)(0, 128), flags=flags)

    B = 8192
    assert lib.tt_tower_workspace_bytes(C.byref(shape(0)), B) > 0
    assert lib.tt_tower_workspace_bytes(C.byref(shape(_lib.TT_TOWER_GENERAL_T1)), B) > 0
    assert lib.tt_tower_workspace_bytes(C.byref(shape(4)), B) == 0
    assert lib.tt_tower_num_params(C.byref(shape(0x100))) == -1
    sh = shape(_lib.TT_TOWER_GENERAL_T1)
    ws = lib.tt_tower_workspace_bytes(C.byref(sh), B)
    fake = 1 << 20  # never dereferenced: the call must return before any launch
    rc = lib.tt_tower_fwd_bwd(C.byref(sh), B, fake, 256, fake, fake, fake, _lib.TT_I32, 1.0, fake, fake, ws, None)
    assert rc == 1001 and b"GENERAL_T1" in lib.tt_last_error_string()


def test_tableset_view_of_maps_shards_onto_shared_storage():
    """ops.TableSet.view_of (the fused sharded step adopting a ShardedEmbeddingBagCollection's
    shards, dropin.FusedShardedDropin): table t of the view is table table_ids[t] of the source —
    same offsets in the same weight / state storage — and a missing shard is a 0-row table."""
    import torch

    from two_tower_recommender_model_amd import ops

    src = ops.TableSet([5, 7, 3], [8, 8, 8], [0, 1, 2], torch.device("cpu"))
    src.weights.copy_(torch.arange(src.weights.numel(), dtype=torch.float32))
    src.state.copy_(torch.arange(src.state.numel(), dtype=torch.float32))
    v = ops.TableSet.view_of(src, [2, None, 0], [8, 8, 8], torch.device("cpu"))
    assert v.rows == [3, 0, 5] and v.weights.data_ptr() == src.weights.data_ptr() and v.state is src.state
    assert torch.equal(v.table_view(0), src.table_view(2)) and torch.equal(v.table_view(2), src.table_view(0))
    assert v.table_view(1).shape == (0, 8) and v.state_view(1).numel() == 0
    assert torch.equal(v.state_view(0), src.state_view(2))
    for t, i in enumerate([2, None, 0]):
        assert v._tm[t].num_rows == (src.rows[i] if i is not None else 0)
        if i is not None:
            assert v._tm[t].weight_offset == src.weight_offsets[i] and v._tm[t].state_offset == src.state_offsets[i]
    # a rank holding no shard at all: empty tables over a one-element storage
    e = ops.TableSet.view_of(None, [None, None], [8, 8], torch.device("cpu"))
    assert e.rows == [0, 0] and e.weights.numel() >= 1
