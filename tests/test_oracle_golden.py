"""Pin the CPU oracle (oracle/torch_ref.py) against golden vectors produced by the reference's
own PyTorch path (tests/golden/make_golden.py).  CPU only."""
import numpy as np
import torch

from conftest import load_case
from oracle import torch_ref as R


def _params(d):
    return R.Params(d["mu"], d["scaling"], d["rotation"], d["opacity"], d["features_dc"],
                    d["features_rest"], d["meta"]["deg"])


def test_units_sh_rotation_pdf():
    u = load_case("units")
    dirs = torch.from_numpy(u["sh_dirs"])
    for deg in range(5):
        out = R.eval_sh(deg, torch.from_numpy(u[f"sh{deg}_coef"]), dirs)
        np.testing.assert_allclose(out.numpy(), u[f"sh{deg}_out"], rtol=1e-6, atol=1e-6)
    Rm = R.build_rotation(torch.from_numpy(u["rot_q"]))
    np.testing.assert_allclose(Rm.numpy(), u["rot_R"], rtol=1e-6, atol=1e-6)

    class P:
        pass
    P._mu = torch.from_numpy(u["pdf_mu"])
    P._scaling = torch.from_numpy(u["pdf_scaling"])
    P._rotation = torch.from_numpy(u["pdf_rotation"])
    x = torch.from_numpy(u["pdf_x"])
    np.testing.assert_allclose(R.gaussian_pdf(x, P, "torch", 1.0).numpy(), u["pdf_out"], rtol=1e-6)
    np.testing.assert_allclose(R.gaussian_pdf(x, P, "torch", 0.7).numpy(), u["pdf_out_mod"], rtol=1e-6)


def test_oracle_matches_reference(golden_case):
    d = golden_case
    m = d["meta"]
    P = _params(d)
    box = torch.from_numpy(d["box"])
    walls = torch.from_numpy(d["walls"])
    Y = float(d["volume_position"][1])
    mode = "netf" if m["occlusion"] else "noocl"
    total = 0.0
    for w in range(m["nwall"]):
        tab = R.sample_tables(walls[w], box, m["ns"], m["start"], m["end"], m["c"], m["deltaT"])
        if w == 0:
            np.testing.assert_array_equal(tab["input_points"].numpy(), d["input_points0"])
        assert tab["I1"] == d["I1"][w] and tab["I2"] == d["I2"][w]
        assert abs(tab["dtheta"] - d["dtheta"][w]) < 1e-12 and abs(tab["dphi"] - d["dphi"][w]) < 1e-12
        result, hist = R.render_wallpoint(P, walls[w], tab, Y, m["c"], m["deltaT"], "torch", mode)
        np.testing.assert_allclose(result.detach().numpy(), d["result"][w], rtol=2e-6, atol=1e-7)
        np.testing.assert_allclose(hist.detach().numpy(), d["hist"][w], rtol=2e-6, atol=1e-6)
        target = torch.from_numpy(d["nlos_data"][tab["I1"]:tab["I1"] + tab["nr"], 0, w]) * m["gt_times"]
        loss, eq = R.mse_loss(hist, target)
        np.testing.assert_allclose(loss.item(), d["loss"][w], rtol=1e-5)
        np.testing.assert_allclose(eq.item(), d["equal_loss"][w], rtol=1e-5)
        total = total + loss
    total.backward()
    for name, leaf in zip(["mu", "scaling", "rotation", "opacity", "features_dc", "features_rest"],
                          P.leaves()):
        ref = d["grad_" + name]
        scale = max(np.abs(ref).max(), 1e-12) if ref.size else 1.0
        np.testing.assert_allclose(leaf.grad.numpy(), ref, rtol=1e-4, atol=1e-5 * scale,
                                   err_msg=name)
