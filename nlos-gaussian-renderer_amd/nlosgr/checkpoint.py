"""Checkpoints with the reference's keys (GaussianModel.get_params / restore, gaussian_model.py:63-103;
written by main.py's save_model) that load with torch.load(weights_only=True).

The reference pickles the torch.optim.Adam object itself under 'optimizer', so its files only load
with weights_only=False. Here 'optimizer' holds an Adam *state_dict* (plain tensors and numbers,
the layout torch.optim.Adam.state_dict() produces for the six groups of gaussian_model.py:229-236),
which the reference's restore accepts through its `load_state_dict(params['optimizer'])` branch,
and which TrainStep reloads into its on-device Adam moments.
"""
import torch

from .model import GaussianParams

PARAM_KEYS = ("mu", "features_dc", "features_rest", "opacity", "scaling", "rotation")
GROUP_ORDER = ("mu", "f_dc", "f_rest", "opacity", "scaling", "rotation")     # gaussian_model.py:229-236


def _group(name, i, lr, betas=(0.9, 0.999), eps=1e-15):
    return {"lr": float(lr), "betas": tuple(betas), "eps": float(eps), "weight_decay": 0.0, "amsgrad": False,
            "maximize": False, "foreach": None, "capturable": False, "differentiable": False, "fused": None,
            "name": name, "params": [i]}


def _adam_state_dict(model, step, spatial_lr_scale=1.0):
    """train.TrainStep's Adam as a torch.optim.Adam state_dict (group order of the reference,
    gaussian_model.py:229-236).  The moments are stored in the shapes of the reference's parameter
    tensors (features_dc [N,1,C], features_rest [N,K-1,C], opacity [N,1]; gaussian_model.py:217-221),
    so the reference's own optimizer.load_state_dict + step accept them; TrainStep keeps flattened
    views of the same tensors.  Without a TrainStep a fresh state (no moments yet) is written, which
    torch.optim.Adam.load_state_dict also accepts; its mu group lr is position_lr_init *
    spatial_lr_scale as training_setup sets it (gaussian_model.py:230), since load_state_dict copies the
    saved group hyperparameters over the live ones."""
    if step is None:
        from .train import OptimizationParams
        o = OptimizationParams()
        lrs = [o.position_lr_init * float(spatial_lr_scale), o.feature_lr, o.feature_lr / 20.0, o.opacity_lr, o.scaling_lr, o.rotation_lr]
        return {"state": {}, "param_groups": [_group(n, i, lrs[i]) for i, n in enumerate(GROUP_ORDER)]}
    adam = step.adam
    lrs = step.learning_rates(step.iteration)
    state, groups = {}, []
    for i, (name, key) in enumerate(zip(GROUP_ORDER, PARAM_KEYS)):
        shape = getattr(model, "_" + key).shape
        state[i] = {"step": torch.tensor(float(adam.step_count)),
                    "exp_avg": adam.exp_avg[i].detach().reshape(shape).cpu().clone(),
                    "exp_avg_sq": adam.exp_avg_sq[i].detach().reshape(shape).cpu().clone()}
        groups.append(_group(name, i, lrs[i], adam.betas, adam.eps))
    return {"state": state, "param_groups": groups}


def save_checkpoint(path, model, train_step=None, spatial_lr_scale=None):
    """torch.save of {mu, features_dc, features_rest, opacity, scaling, rotation, optimizer,
    max_sh_degree, active_sh_degree} (+ 'iteration' when a TrainStep is given).  spatial_lr_scale
    (default: the TrainStep's, else the model's attribute, else 1) scales the fresh mu group lr."""
    if spatial_lr_scale is None:
        spatial_lr_scale = getattr(train_step, "spatial_lr_scale", None) or getattr(model, "spatial_lr_scale", 1.0)
    ck = {k: getattr(model, "_" + k).detach().cpu() for k in PARAM_KEYS}
    ck["max_sh_degree"] = int(model.max_sh_degree)
    ck["active_sh_degree"] = int(model.active_sh_degree)
    ck["optimizer"] = _adam_state_dict(model, train_step, spatial_lr_scale)
    if train_step is not None:
        ck["iteration"] = int(train_step.iteration)
    torch.save(ck, path)


def load_checkpoint(path, device="cpu", train_step=None):
    """GaussianParams from a checkpoint (weights_only=True: a reference file with a pickled optimizer
    object is refused by torch; re-save it with the optimizer as a state_dict).  With train_step,
    its parameters, Adam moments, step count and iteration are restored in place."""
    ck = torch.load(path, map_location="cpu", weights_only=True)
    t = {k: ck[k].float().to(device) for k in PARAM_KEYS}
    model = GaussianParams(t["mu"], t["scaling"], t["rotation"], t["opacity"], t["features_dc"], t["features_rest"],
                           int(ck["active_sh_degree"]), int(ck["max_sh_degree"]))
    if train_step is not None:
        m = train_step.model
        with torch.no_grad():
            for k in PARAM_KEYS:
                getattr(m, "_" + k).data.copy_(t[k].to(m._mu.device))
        m.active_sh_degree = int(ck["active_sh_degree"])
        opt = ck.get("optimizer")
        if opt and opt.get("state"):
            for i in range(len(GROUP_ORDER)):
                st = opt["state"][i]
                train_step.adam.exp_avg[i].copy_(st["exp_avg"].reshape(train_step.adam.exp_avg[i].shape))
                train_step.adam.exp_avg_sq[i].copy_(st["exp_avg_sq"].reshape(train_step.adam.exp_avg_sq[i].shape))
            train_step.adam.step_count = int(float(opt["state"][0]["step"]))
        train_step.iteration = int(ck.get("iteration", train_step.iteration))
    return model
