"""The reference's whole-module checkpoints, read weights-only.

The reference saves and loads entire pickled modules
(``torch.save(model, ...)``; ``torch.load(cp_filename)`` at models.py:421 /
:1076), e.g. the shipped ``outputs/pre_training_v1_GIN_64_5_1.pt``.  Such a
file names the reference's classes (``models.Mainmodel_continue``,
``dgl...GINConv``, ...), so a plain weights-only load refuses it.  Here it is
read with ``torch.load(weights_only=True)`` and, allow-listed through
``torch.serialization.safe_globals``, inert stand-in classes of this module
that carry those names: the restricted unpickler builds each stand-in with
``__new__`` and fills its ``__dict__`` from the file's state — nothing from
the file is executed and no reference module is imported.  The parameters
and persistent buffers are then collected from the stand-ins' ``_parameters``
/ ``_buffers`` / ``_modules`` into a state_dict (544 tensors for the shipped
checkpoint), and the model is rebuilt from this package's classes
(``models.load_checkpoint``).

A file that names any class outside ``_STANDINS`` is refused (the pickle's
global references are listed with ``pickletools``, a disassembler, before
anything is loaded).
"""
from __future__ import annotations

import io
import pickletools
import zipfile

import torch

# every class the reference's pretraining checkpoints reference (besides the
# tensor-rebuild globals torch's weights-only unpickler already allows)
_STANDINS = (
    "models.GIN", "models.MLP", "models.Mainmodel", "models.Mainmodel_continue",
    "models.Mainmodel_domainadapt", "models.Mainmodel_finetuning",
    "dgl.nn.pytorch.conv.ginconv.GINConv", "dgl.nn.pytorch.glob.Set2Set",
    "torch.nn.modules.activation.ReLU", "torch.nn.modules.batchnorm.BatchNorm1d",
    "torch.nn.modules.container.ModuleList", "torch.nn.modules.container.Sequential",
    "torch.nn.modules.linear.Linear", "torch.nn.modules.rnn.LSTM",
)
_TORCH_OK = {"collections.OrderedDict", "torch.FloatStorage", "torch.LongStorage",
             "torch.device", "torch._utils._rebuild_parameter",
             "torch._utils._rebuild_tensor_v2", "__builtin__.set", "builtins.set"}
MODEL_KINDS = ("Mainmodel", "Mainmodel_continue", "Mainmodel_domainadapt")


class RefCheckpointError(RuntimeError):
    pass


def _standin(full):
    mod, _, name = full.rpartition(".")
    cls = type(name, (), {"__module__": mod, "__doc__": f"inert stand-in for {full}"})
    cls.__qualname__ = name
    return cls


def pickle_globals(path):
    """Fully qualified names of every global the checkpoint's pickle
    references (disassembled, not loaded)."""
    with zipfile.ZipFile(path) as z:
        pk = [n for n in z.namelist() if n.endswith("data.pkl")]
        if len(pk) != 1:
            raise RefCheckpointError(f"{path}: not a torch zip checkpoint")
        data = z.read(pk[0])
    # STACK_GLOBAL takes module and name from the stack: they are the two
    # values pushed just before it, each a unicode literal or a memo fetch of
    # one (BINGET after MEMOIZE / BINPUT).  Every other opcode is recorded as an
    # unknown value, so a STACK_GLOBAL whose operands cannot be resolved here
    # is refused rather than misnamed.
    out, pushed, memo = set(), [], {}
    for op, arg, _ in pickletools.genops(io.BytesIO(data)):
        name = op.name
        if name in ("SHORT_BINUNICODE", "BINUNICODE", "UNICODE", "BINUNICODE8"):
            pushed.append(arg)
        elif name == "MEMOIZE":
            memo[len(memo)] = pushed[-1] if pushed else None
        elif name in ("PUT", "BINPUT", "LONG_BINPUT"):
            memo[arg] = pushed[-1] if pushed else None
        elif name in ("GET", "BINGET", "LONG_BINGET"):
            pushed.append(memo.get(arg))
        elif name == "GLOBAL":
            out.add(arg.replace(" ", "."))
            pushed.append(None)
        elif name == "STACK_GLOBAL":
            mod, nm = (pushed[-2], pushed[-1]) if len(pushed) >= 2 else (None, None)
            if not (isinstance(mod, str) and isinstance(nm, str)):
                raise RefCheckpointError(f"{path}: a STACK_GLOBAL whose module / name are not "
                                         "string literals or memo references to them; refused")
            out.add(f"{mod}.{nm}")
            pushed.append(None)
        else:
            pushed.append(None)
    return out


def is_reference_module_checkpoint(path):
    """True for a whole-module pickle of the reference's model classes."""
    try:
        return any(g.startswith("models.Mainmodel") for g in pickle_globals(path))
    except (OSError, zipfile.BadZipFile, RefCheckpointError, ValueError):
        return False


def _kind(obj):
    return type(obj).__name__


def _state(obj, prefix=""):
    d = obj.__dict__
    skip = d.get("_non_persistent_buffers_set") or set()
    for k, v in (d.get("_parameters") or {}).items():
        if v is not None:
            yield prefix + k, v
    for k, v in (d.get("_buffers") or {}).items():
        if v is not None and k not in skip:
            yield prefix + k, v
    for k, m in (d.get("_modules") or {}).items():
        if m is not None:
            yield from _state(m, prefix + k + ".")


def read(path):
    """(kinds, config, state_dict) of a reference whole-module checkpoint.

    kinds: the wrapper chain from the root, one (kind, F) per level (the
    shipped file: Mainmodel_continue x 3 around a Mainmodel — pretraining
    continued over PCQM4Mv2, QM9 and mol-PCBA — each level with its own
    transfer_d input width F); config: the sizes shared by all levels
    (hidden, k, GIN depth, head width, the root's args-derived attributes);
    state_dict: detached CPU tensors."""
    names = pickle_globals(path)
    unknown = {g for g in names if g not in _STANDINS and g not in _TORCH_OK}
    if unknown:
        raise RefCheckpointError(f"{path}: references classes outside the known set: "
                                 f"{sorted(unknown)}")
    standins = [_standin(g) for g in _STANDINS if g in names]
    with torch.serialization.safe_globals(standins + [set]):
        root = torch.load(path, map_location="cpu", weights_only=True)
    if _kind(root) not in MODEL_KINDS or not hasattr(root, "__dict__"):
        raise RefCheckpointError(f"{path}: root object is {_kind(root)}, not a model")
    sd = {k: v.detach().clone() if isinstance(v, torch.Tensor) else v for k, v in _state(root)}
    kinds, m, prefix = [], root, ""
    while m is not None and _kind(m) in MODEL_KINDS:
        kinds.append((_kind(m), int(sd[prefix + "transfer_d.weight"].shape[1])))
        m = (m.__dict__.get("_modules") or {}).get("model")
        prefix += "model."
    if not kinds:
        raise RefCheckpointError(f"{path}: root object is {_kind(root)}, not a model")
    attrs = root.__dict__
    gin = [k for k in sd if k.startswith("Encoder1.ginlayers.") and k.endswith("apply_func.mlp.0.weight")]
    pred = sd.get("predict.2.weight")
    cfg = {
        "kinds": kinds,
        "in_dim": int(sd["transfer_d.weight"].shape[1]),
        "d_transfer": int(sd["transfer_d.weight"].shape[0]),
        "hidden_dim": int(attrs.get("hidden_dim", 64)),
        "k_transition": int(attrs.get("k_transition", 1)),
        "gin_layers": len(gin),
        "num_classes": int(pred.shape[0]) if pred is not None else 1,
        "recons_type": attrs.get("recons_type", "adj"),
        "useAtt": int(attrs.get("useAtt", 1)),
        "readout_f": attrs.get("readout", "sum"),
        "batch_size": int(attrs.get("batch_size", 16)),
    }
    return kinds, cfg, sd
