"""Path options of the Python host (the library's own kernel-path options are vs_set_option,
`kernels.set_option`).  One table, product defaults; tests and A/B probes select the others with
`set_host_option` / the `host_options(...)` context manager, and whole runs with the one environment
hook VSTYLER_OPTS="sp_comm=native,sp_graph=1,queue=0" (host names here, every other name a library
option), read once when the package is imported.

  sp_overlap      1      Ulysses: split the CFG batch into per-sample micro-batches so one sample's
                         all-to-alls run under the other's compute (usp.UlyssesGroup)
  sp_comm         torch  Ulysses / CFG-parallel collectives: "torch" (torch.distributed's RCCL) or
                         "native" (libvstyler's vs_sp_* communicator, usp.NativeComm)
  sp_comm_stream  side   NativeComm: collectives on a stream of their own ("side") or the caller's
  sp_graph        0      capture the SP step's collectives into the step's hipGraph (native comm only;
                         pipeline.sp_graph_ok)
  sp_rows         1      batch-1 exchanges deliver q|k|v rows in token order (no re-layout)
  sp_merge_ffn    1      Ulysses overlap: phase 4 (cross-attention + FFN) over both samples' rows at once
  cfg_parallel    0      "0" Ulysses over all ranks, "1" CFG parallelism x Ulysses, "auto" CFG
                         parallelism at world size 2 only (usp.get_default_group)
  fuse_res_ln     1      the residual + LayerNorm fused into the producing GEMM's consumer (models)
  fuse_ffn_ln     1      the next block's LN1 fused after the FFN-down epilogue (models)
  ws_poison       0      Workspace fills every fresh buffer with NaN (debugging stale reads)
  graph           1      hipGraph replay of the denoising step (pipeline.WanVideoPipeline.denoise)
  cfg_prefix      1      the first DiT block's and the first VACE block's phases 1-3 (LN1, q|k|v,
                         self-attention, o-proj, LN3) run once for both CFG samples when their rows are
                         equal (shared latents / timestep / VACE context): bit-identical (DiTBlock)
"""
HOST_DEFAULTS = {
    "sp_overlap": 1, "sp_comm": "torch", "sp_comm_stream": "side", "sp_graph": 0, "sp_rows": 1,
    "sp_merge_ffn": 1, "cfg_parallel": "0", "fuse_res_ln": 1, "fuse_ffn_ln": 1, "ws_poison": 0, "graph": 1,
    "cfg_prefix": 1,
}
_CHOICES = {"sp_comm": ("torch", "native"), "sp_comm_stream": ("side", "caller"),
            "cfg_parallel": ("0", "1", "auto")}
_HOST = dict(HOST_DEFAULTS)


def _coerce(name, value):
    if name not in HOST_DEFAULTS:
        raise KeyError(f"unknown host option {name!r} (known: {', '.join(HOST_DEFAULTS)})")
    if name in _CHOICES:
        value = str(value)
        if value not in _CHOICES[name]:
            raise ValueError(f"host option {name} must be one of {_CHOICES[name]}, not {value!r}")
        return value
    return int(value)


def host_option(name):
    if name not in _HOST:
        raise KeyError(f"unknown host option {name!r}")
    return _HOST[name]


def set_host_option(name, value):
    """Set a host option; returns the previous value."""
    value = _coerce(name, value)
    prev = _HOST[name]
    _HOST[name] = value
    return prev


class host_options:
    """Context manager: host_options(sp_merge_ffn=0, sp_graph=1) for the duration of a with-block."""

    def __init__(self, **kw):
        self.kw, self.saved = kw, {}

    def __enter__(self):
        for k, v in self.kw.items():
            self.saved[k] = set_host_option(k, v)
        return self

    def __exit__(self, *exc):
        for k, v in self.saved.items():
            set_host_option(k, v)
        return False


def apply_spec(spec, set_library_option=None):
    """VSTYLER_OPTS syntax: comma-separated name=value; host names set here, the rest through
    `set_library_option` (kernels.set_option)."""
    for item in filter(None, (x.strip() for x in spec.split(","))):
        name, _, value = item.partition("=")
        name = name.strip()
        if name in HOST_DEFAULTS:
            set_host_option(name, value.strip())
        elif set_library_option is not None:
            set_library_option(name, int(value))
        else:
            raise KeyError(f"unknown host option {name!r}")
