"""CPU checks of the decode-GEMM router's gemm_xd forms and of the in-tree tuning table
(ops/gemm.py; no GPU work: forms are parsed and shape-checked on the host)."""
import json

import pytest

from drtc_amd.ops import gemm as G


def test_xd_form_parsing():
    assert G.xd_form(244) == (2, 4, 4) and not G.xd_nt(244)
    assert G.xd_form(1244) == (2, 4, 4) and G.xd_nt(1244)
    assert G.xd_form(1281) == (2, 8, 1)


def test_nontemporal_forms_only_for_built_tiles():
    assert G.xd_supported(256, 8192, 28672, 1244)
    assert G.xd_supported(256, 28672, 8192, 1281, glu=True)
    assert not G.xd_supported(256, 1536, 2048, 1121)  # 128 x 64: no non-temporal build
    assert not G.xd_supported(256, 1536, 2048, 2244)  # not a form


@pytest.mark.parametrize("M,form,want", [
    (256, 244, 1244),   # one 256-row tile: every weight byte read once
    (128, 141, 1141),
    (160, 141, 141),    # two 128-row tiles share the weight panel through L2
    (1024, 281, 281),
    (256, 121, 121),    # 128 x 64 tile: no non-temporal build
    (256, 1243, 1243),  # tuned non-temporal form: as tuned
    (512, 0, 0),
])
def test_router_policy_picks_nontemporal_twin(monkeypatch, M, form, want):
    monkeypatch.setattr(G, "_xd_nt", True)
    monkeypatch.setattr(G, "_xd_enabled", True)
    assert G._xd_policy(M, form) == want
    monkeypatch.setattr(G, "_xd_nt", False)
    assert G._xd_policy(M, form) == form % 1000  # DRTC_XD_NT=0: every form plain
    monkeypatch.setattr(G, "_xd_enabled", False)
    assert G._xd_policy(M, form) == 0


def test_router_keeps_nt_tuned_plain_winner(monkeypatch):
    """An entry the nt-aware re-tune measured (profiles/r4ab: Llama-3-8B gate_up at M = 160-256
    picked plain 241 over 1241) runs exactly its pick; its nt picks stay nt unless
    DRTC_XD_NT=0; the committed table marks those entries."""
    monkeypatch.setattr(G, "_xd_enabled", True)
    monkeypatch.setattr(G, "_xd_nt", True)
    assert G._xd_policy(160, 241, nt_tuned=True) == 241
    assert G._xd_policy(160, 241, nt_tuned=False) == 1241
    assert G._xd_policy(256, 1244, nt_tuned=True) == 1244
    monkeypatch.setattr(G, "_xd_nt", False)
    assert G._xd_policy(256, 1244, nt_tuned=True) == 244
    with open(G.table_path()) as f:
        data = json.load(f)
    e = next(iter(data.values()))["160,28672,4096,4096"]
    assert e["xd"] == 241 and e["nt_tuned"]


def test_every_tuned_xd_form_fits_its_shape():
    """Each xd / xd_glu entry of the committed table names a built form that takes its own
    shape (what the router would run, including the non-temporal twin)."""
    with open(G.table_path()) as f:
        data = json.load(f)
    n = 0
    for entries in data.values():
        for key, e in entries.items():
            M, N, K, _ = (int(v) for v in key.split(","))
            if e.get("xd"):
                n += 1
                assert G.xd_supported(M, N, K, e["xd"]), (key, e["xd"])
                assert G.xd_supported(M, N, K, G._xd_policy(M, e["xd"]) or e["xd"]), key
            if e.get("xd_glu"):
                n += 1
                assert N % 2 == 0
                assert G.xd_supported(M, N // 2, K, e["xd_glu"], glu=True), (key, e["xd_glu"])
    assert n > 100


def test_gemma_2048_decode_shapes_carry_a_gemm_xd_form():
    """Gemma-2B's 2,048-row decode batch (above the 1,024 decode buckets): the tuned table
    gives its qkv / o / down shapes a gemm_xd form next to their prefill library entries
    (profiles/r6ak), and every such form fits its shape."""
    tab = json.load(open(G.table_path()))
    for ver, ents in tab.items():
        for k, want in (("2048,2560,2048,2048", 241), ("2048,2048,2048,2048", 141),
                        ("2048,2048,16384,16384", 242)):
            e = ents.get(k)
            if e is None:
                continue
            assert e.get("prefill") and e["xd"] == want
            M, N, K, _ = (int(v) for v in k.split(","))
            assert G.xd_supported(M, N, K, want)
