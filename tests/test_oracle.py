"""The oracle (CPU restatement) pinned against the reference's own outputs (golden fixtures)."""
import numpy as np
import pytest
import torch

from conftest import golden
from helpers import batch_from_fixture, oracle_model, rel_err

from oracle import ref_cpu, triplets


def test_triplets_match_reference_all_cases():
    z = golden("triplets.npz")
    for case in z["cases"]:
        ei, n = z[f"{case}_edge_index"], int(z[f"{case}_num_nodes"])
        trip, j, i, k = triplets.vertex_to_edge(ei, n)
        np.testing.assert_array_equal(trip, z[f"{case}_trip"])
        np.testing.assert_array_equal(j, z[f"{case}_j"])
        np.testing.assert_array_equal(i, z[f"{case}_i"])
        np.testing.assert_array_equal(k, z[f"{case}_k"])


def test_triplets_brute_force_small_cases():
    z = golden("triplets.npz")
    for case in ("s160", "directed"):
        ei, n = z[f"{case}_edge_index"], int(z[f"{case}_num_nodes"])
        trip, j, i, k = triplets.brute_force(ei, n)
        np.testing.assert_array_equal(trip, z[f"{case}_trip"])
        np.testing.assert_array_equal(k, z[f"{case}_k"])


def test_triplet_count_known_answer():
    from x2gnn.synth import triplet_count

    z = golden("triplets.npz")
    for case in z["cases"]:
        ei, n = z[f"{case}_edge_index"], int(z[f"{case}_num_nodes"])
        assert triplet_count(ei, n) == z[f"{case}_trip"].shape[1]
        if case != "directed":  # symmetric graphs: T = sum_b deg(b)(deg(b)-1)
            deg = np.bincount(ei[0], minlength=n)
            assert (deg * (deg - 1)).sum() == z[f"{case}_trip"].shape[1]


def test_envelope_known_answers():
    z = golden("basis.npz")
    np.testing.assert_allclose(ref_cpu.envelope(torch.from_numpy(z["env_probe_d"])).numpy(), z["env_probe"],
                               rtol=1e-6, atol=1e-5)
    assert abs(float(ref_cpu.envelope(torch.tensor(5.0)))) < 1e-5  # 1 - 28 + 48 - 21 = 0


def test_basis_constants_known_answers():
    assert np.allclose(ref_cpu._basis_consts(7, 6)[0][0], np.pi * np.arange(1, 7), rtol=1e-7)   # z_0n = n pi
    y = ref_cpu.sph_y0(np.array([0.3]))
    assert abs(y[0, 0] - 1 / (2 * np.sqrt(np.pi))) < 1e-12                      # Y_00 = 1/(2 sqrt(pi))


def test_spherical_basis_vs_reference():
    z = golden("basis.npz")
    sbf = ref_cpu.spherical_basis(torch.from_numpy(z["dist"]), torch.from_numpy(z["theta"]),
                                  torch.from_numpy(z["trip"][0].astype(np.int64))).numpy()
    ref = z["sbf"]
    # the reference's fp32 expanded j_l loses digits at small d (cancellation grows with l):
    # compare column blocks l with an l-dependent absolute tolerance, plus a global relative bound
    for l in range(7):
        blk = slice(6 * l, 6 * l + 6)
        tol = [1e-5, 1e-5, 1e-5, 1e-4, 1e-3, 5e-3, 3e-2][l]
        assert np.abs(sbf[:, blk] - ref[:, blk]).max() < tol, l
    assert rel_err(sbf, ref) < 2e-2


def test_conv_layer_vs_reference():
    z = golden("conv1.npz")
    from weights import load_seeded

    conv = ref_cpu.SBFTransformerConv(128, 16, 42, 6, 128)
    load_seeded(conv, int(z["weight_seed"]))
    x = torch.from_numpy(z["conv_x"]).requires_grad_(True)
    ea = torch.from_numpy(z["conv_edge_attr"]).requires_grad_(True)
    out = conv(torch.from_numpy(z["sbf"]), torch.from_numpy(z["rbf"]), x,
               torch.from_numpy(z["trip"].astype(np.int64)), ea)
    assert rel_err(out.detach().numpy(), z["out"]) < 1e-5
    (out * torch.from_numpy(z["upstream"])).sum().backward()
    assert rel_err(x.grad.numpy(), z["grad_x"]) < 1e-4
    assert rel_err(ea.grad.numpy(), z["grad_edge_attr"]) < 1e-4
    for n, p in conv.named_parameters():
        assert rel_err(p.grad.numpy(), z["grad." + n]) < 1e-4, n


@pytest.mark.parametrize("fixture", ["model_small.npz", "model_full.npz", "model_global.npz", "model_s5a.npz",
                                     "model_global_add.npz", "model_aid.npz", "model_s5a_full.npz"])
def test_model_vs_reference(fixture):
    z = golden(fixture)
    m = oracle_model(z)
    b = batch_from_fixture(z)
    res = ref_cpu.run_batch(m, b)
    assert rel_err(res.detach().numpy(), z["energies"]) < 1e-4
    loss = torch.nn.functional.smooth_l1_loss(res, b.y)
    loss.backward()
    np.testing.assert_allclose(m.emb_block.embedding.weight.detach().numpy(), z["emb_after"], rtol=1e-6, atol=1e-7)
    # gradients that vanish analytically (e.g. lin_key.bias: softmax is shift invariant) are
    # rounding noise on both sides, so the absolute slack scales with the largest gradient
    scale = max(float(z["gnorm." + n]) for n, _ in m.named_parameters())
    for n, p in m.named_parameters():
        ref_norm = float(z["gnorm." + n])
        got = 0.0 if p.grad is None else float(p.grad.double().norm())
        assert abs(got - ref_norm) <= 1e-3 * ref_norm + 1e-6 * scale, (n, got, ref_norm)
        if "grad." + n in z.files:
            ref = z["grad." + n]
            assert np.abs(p.grad.numpy() - ref).max() <= 2e-3 * np.abs(ref).max() + 1e-6 * scale, n


def test_spherical_basis_7x16_vs_reference():
    """The oracle's F_B_2D(7, 16) (the reference's default basis, xgnn.py:16) against the
    reference's own fp32 output: within 1e-4 (the reference's fp32 expansion vs fp64 scipy)."""
    z = golden("basis_7x16.npz")
    sbf = ref_cpu.spherical_basis(torch.from_numpy(z["dist"]), torch.from_numpy(z["theta"]),
                                  torch.from_numpy(z["trip"][0].astype(np.int64)), 7, 16).numpy()
    assert sbf.shape == z["sbf"].shape
    assert np.abs(sbf - z["sbf"]).max() < 1e-4
