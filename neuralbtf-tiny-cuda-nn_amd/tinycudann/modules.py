"""torch.nn front-end mirroring reference bindings/torch/tinycudann/modules.py:91-329 on top of the
C-ABI runtime module (include/tcnn_mi355x.h, which replaces reference src/cpp_api.cu +
bindings/torch/tinycudann/bindings.cpp).

Provenance: the autograd plumbing below (null-tensor conventions, `_module_function`,
`_module_function_backward`, `Module.forward`'s batch padding and the pickling hooks) follows the
reference's modules.py:81-204 (tiny-cuda-nn, Copyright (c) 2020-2022 NVIDIA CORPORATION, BSD-3-Clause)
closely on purpose: it is the plugin API whose exact behaviour -- loss-scale multiply/divide order,
null-tensor conventions, output slicing -- callers such as NeuralBTF depend on."""
import ctypes
import gc
import json
import os
import sys
import warnings

import torch

from tinycudann import _lib as L

if not torch.cuda.is_available():
    raise EnvironmentError("Unknown compute capability. Ensure PyTorch with ROCm support and an MI355X are available.")

PRECISION_FP32 = 0
PRECISION_FP16 = 1


class _C:
    """Stand-in for the reference's compiled `tinycudann._C` module-level functions
    (bindings.cpp:285-336), so scripts written against it (e.g. scripts/test_grid_bwdbwd.py,
    which imports `_C` from tinycudann.modules) run unchanged. Everything goes to the C-ABI."""

    class Precision:
        Fp32 = PRECISION_FP32
        Fp16 = PRECISION_FP16

    @staticmethod
    def preferred_precision():
        return L.lib().tcnn_preferred_precision()

    @staticmethod
    def batch_size_granularity():
        return L.lib().tcnn_batch_size_granularity()

    @staticmethod
    def default_loss_scale(precision):
        return L.lib().tcnn_default_loss_scale(precision)

    @staticmethod
    def free_temporary_memory():
        L.lib().tcnn_free_temporary_memory()

    @staticmethod
    def has_networks():
        return bool(L.lib().tcnn_has_networks())


def _torch_precision(p):
    return torch.half if p == PRECISION_FP16 else torch.float


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def _stream(t=None):
    """the current stream of t's device (default: the current device) as a raw handle -- the binding's
    hot path makes a few of these calls per step, and torch.cuda.current_stream() builds a Stream object
    each time (the torch step is host-bound at 2^16 points, tools/torch_host_breakdown.py)"""
    if _raw_stream is not None:
        return _raw_stream(t.device.index if t is not None else torch.cuda.current_device())
    return torch.cuda.current_stream().cuda_stream


def _ptr(t):
    return t.data_ptr() if t is not None else None  # ctypes converts the int for a c_void_p argument


_GRANULARITY = None

# The C++ autograd node (csrc/torch_ext.cpp, built in-tree next to the engine library): one pybind call per
# forward and a C++ backward. The Python autograd.Function below is the same node and stays the fallback
# (TCNN_TORCH_PY=1 selects it: A/B switch).
_EXT = None
if not os.environ.get("TCNN_TORCH_PY"):
    try:
        _libdir = os.path.dirname(L.LIB_PATH)
        if _libdir not in sys.path:
            sys.path.append(_libdir)
        import _tcnn_torch as _EXT  # noqa: E402
    except ImportError:
        _EXT = None


def _granularity():
    global _GRANULARITY
    if _GRANULARITY is None:
        _GRANULARITY = int(L.lib().tcnn_batch_size_granularity())
    return _GRANULARITY


def free_temporary_memory():
    gc.collect()
    L.lib().tcnn_free_temporary_memory()


class _NativeModule:
    """Python twin of bindings.cpp's Module class (bindings.cpp:75-171). A module's sizes and
    precisions are fixed at creation; they are read once here, so a training step makes no ctypes
    round trips for them (the torch step is host-bound: tools/torch_step_profile.py)."""

    def __init__(self, handle):
        self.h = L.check_ptr(handle)
        lib = L.lib()
        self._n_in = lib.tcnn_module_n_input_dims(self.h)
        self._n_out = lib.tcnn_module_n_output_dims(self.h)
        self._n_params = lib.tcnn_module_n_params(self.h)
        self._param_dtype = _torch_precision(lib.tcnn_module_param_precision(self.h))
        self._out_dtype = _torch_precision(lib.tcnn_module_output_precision(self.h))

    # bindings.cpp:306-313: sizes are methods on the native module, as in the reference
    def n_input_dims(self):
        return self._n_in

    def n_output_dims(self):
        return self._n_out

    def n_params(self):
        return self._n_params

    def __del__(self):
        try:
            L.lib().tcnn_module_destroy(self.h)
        except Exception:
            pass

    def param_precision(self):
        return L.lib().tcnn_module_param_precision(self.h)

    def output_precision(self):
        return L.lib().tcnn_module_output_precision(self.h)

    def hyperparams(self):
        return json.loads(L.lib().tcnn_module_hyperparams(self.h).decode())

    def name(self):
        return L.lib().tcnn_module_name(self.h).decode()

    def engine(self):
        """the engine training / backward runs on ("fused", "layered"; "encoding" for encodings)"""
        return L.lib().tcnn_module_engine(self.h).decode()

    def inference_engine(self):
        return L.lib().tcnn_module_inference_engine(self.h).decode()

    def initial_params(self, seed):
        p = torch.zeros(self.n_params(), dtype=torch.float32, device="cuda")
        torch.cuda.synchronize()
        L.check(L.lib().tcnn_module_initialize_params(self.h, seed, _ptr(p), 1.0))
        return p

    def fwd(self, input, params):
        assert input.dtype == torch.float32 and input.is_contiguous() and input.shape[1] == self._n_in
        assert params.dtype == self._param_dtype and params.numel() == self._n_params
        B = input.shape[0]
        out = torch.empty(B, self._n_out, dtype=self._out_dtype, device=input.device)
        if not (input.requires_grad or params.requires_grad):
            L.check(L.lib().tcnn_module_inference(self.h, _stream(input), B, _ptr(input), _ptr(out), _ptr(params)))
            return None, out
        ctx = L.check_ptr(L.lib().tcnn_module_forward(self.h, _stream(input), B, _ptr(input), _ptr(out), _ptr(params),
                                                       int(input.requires_grad)))
        return _NativeContext(ctx), out

    def bwd_scaled(self, ctx, input, params, output, doutput, loss_scale, need_input, need_params):
        """the binding's first-order backward (modules.py:128-138 of the reference: doutput * loss_scale,
        Module::backward, dL/dinput and dL/dparams divided by loss_scale) as ONE engine call
        (tcnn_module_backward_scaled), with the same roundings as the three torch operations"""
        B = input.shape[0]
        dL_dinput = torch.empty_like(input) if need_input else None
        dL_dparams = torch.empty(self._n_params, dtype=self._param_dtype, device=input.device) if need_params else None
        if doutput.dtype != self._out_dtype:
            doutput = doutput.to(self._out_dtype)
        if not doutput.is_contiguous():
            doutput = doutput.contiguous()
        L.check(L.lib().tcnn_module_backward_scaled(self.h, _stream(input), ctx.h, B, _ptr(dL_dinput), _ptr(doutput),
                                                    _ptr(dL_dparams), _ptr(input), _ptr(output), _ptr(params),
                                                    float(loss_scale), 0))
        return dL_dinput, dL_dparams

    def bwd(self, ctx, input, params, output, dL_doutput):
        B = input.shape[0]
        dL_dinput = torch.empty_like(input) if input.requires_grad else None
        dL_dparams = torch.empty(self.n_params(), dtype=_torch_precision(self.param_precision()), device=input.device) if params.requires_grad else None
        dL_doutput = dL_doutput.to(_torch_precision(self.output_precision())).contiguous()
        L.check(L.lib().tcnn_module_backward(self.h, _stream(), ctx.h, B, _ptr(dL_dinput), _ptr(dL_doutput),
                                             _ptr(dL_dparams), _ptr(input), _ptr(output), _ptr(params)))
        return dL_dinput, dL_dparams

    def bwd_bwd_input(self, ctx, input, params, dL_ddLdinput, dL_doutput):
        """bindings.cpp:185-239: second-order gradients from dL/d(dL/dinput)."""
        B = input.shape[0]
        dev = input.device
        dL_ddLdoutput = (torch.zeros(B, self.n_output_dims(), dtype=_torch_precision(self.output_precision()), device=dev)
                         if dL_doutput.requires_grad else None)
        dL_dparams = (torch.zeros(self.n_params(), dtype=_torch_precision(self.param_precision()), device=dev)
                      if params.requires_grad else None)
        dL_dinput = torch.zeros(B, self.n_input_dims(), dtype=torch.float32, device=dev) if input.requires_grad else None
        if dL_doutput.requires_grad or params.requires_grad:
            dL_ddLdinput = dL_ddLdinput.to(torch.float32).contiguous()
            dout = dL_doutput.detach().to(_torch_precision(self.output_precision())).contiguous()
            L.check(L.lib().tcnn_module_backward_backward_input(
                self.h, _stream(), ctx.h, B, _ptr(dL_ddLdinput), _ptr(input),
                _ptr(dout) if (params.requires_grad or input.requires_grad) else None,
                _ptr(dL_dparams), _ptr(dL_ddLdoutput), _ptr(dL_dinput), _ptr(params)))
        return dL_ddLdoutput, dL_dparams, dL_dinput


class _NativeContext:
    def __init__(self, h):
        self.h = h

    def __del__(self):
        try:
            L.lib().tcnn_context_destroy(self.h)
        except Exception:
            pass


def null_tensor_like(tensor):
    return torch.empty([], dtype=tensor.dtype, device=tensor.device)


def null_tensor_to_none(tensor):
    if len(tensor.shape) == 0:
        return None
    return tensor


class _module_function(torch.autograd.Function):
    @staticmethod
    def forward(ctx, native_tcnn_module, input, params, loss_scale):
        ctx.set_materialize_grads(False)
        native_ctx, output = native_tcnn_module.fwd(input, params)
        ctx.save_for_backward(input, params, output)
        ctx.native_tcnn_module = native_tcnn_module
        ctx.native_ctx = native_ctx
        ctx.loss_scale = loss_scale
        return output

    @staticmethod
    def backward(ctx, doutput):
        if doutput is None:
            return None, None, None, None
        if not doutput.is_cuda:
            warnings.warn("doutput must be a CUDA tensor, but isn't. This indicates suboptimal performance.")
            doutput = doutput.cuda()
        input, params, output = ctx.saved_tensors
        if not torch.is_grad_enabled():
            # a first-order backward (no create_graph): nothing will differentiate the gradients, so the
            # differentiable wrapper below and its torch scaling ops are skipped -- one engine call, same values
            if doutput.dtype != output.dtype:
                doutput = doutput.to(output.dtype)  # the binding's doutput * loss_scale has the output's dtype
            input_grad, params_grad = ctx.native_tcnn_module.bwd_scaled(
                ctx.native_ctx, input, params, output, doutput, ctx.loss_scale, ctx.needs_input_grad[1], ctx.needs_input_grad[2])
            return None, input_grad, params_grad, None
        input_grad, params_grad = _module_function_backward.apply(ctx, doutput, input, params, output)
        return None, null_tensor_to_none(input_grad), null_tensor_to_none(params_grad), None


class _module_function_backward(torch.autograd.Function):
    """modules.py:128-170 of the reference: the backward as a differentiable function, so that
    d(dL/dinput)/d(doutput, params, input) flows through Module.bwd_bwd_input."""

    @staticmethod
    def forward(ctx, ctx_fwd, doutput, input, params, output):
        ctx.ctx_fwd = ctx_fwd
        ctx.save_for_backward(input, params, doutput)
        with torch.no_grad():
            scaled_grad = doutput * ctx_fwd.loss_scale
            input_grad, params_grad = ctx_fwd.native_tcnn_module.bwd(ctx_fwd.native_ctx, input, params, output, scaled_grad)
            input_grad = null_tensor_like(input) if input_grad is None else (input_grad / ctx_fwd.loss_scale)
            params_grad = null_tensor_like(params) if params_grad is None else (params_grad / ctx_fwd.loss_scale)
        return input_grad, params_grad

    @staticmethod
    def backward(ctx, dinput_grad, dparams_grad):
        input, params, doutput = ctx.saved_tensors
        if dinput_grad is None:
            return None, None, None, None, None
        with torch.enable_grad():
            doutput = doutput * ctx.ctx_fwd.loss_scale
        with torch.no_grad():
            doutput_grad, params_grad, input_grad = ctx.ctx_fwd.native_tcnn_module.bwd_bwd_input(
                ctx.ctx_fwd.native_ctx, input, params, dinput_grad, doutput)
            params_grad = None if params_grad is None else (params_grad / ctx.ctx_fwd.loss_scale)
            input_grad = None if input_grad is None else (input_grad / ctx.ctx_fwd.loss_scale)
        return None, doutput_grad, input_grad, params_grad, None


class Module(torch.nn.Module):
    def __init__(self, seed=1337):
        super().__init__()
        self.native_tcnn_module = self._native_tcnn_module()
        self.dtype = _torch_precision(self.native_tcnn_module.param_precision())
        self.seed = seed
        initial_params = self.native_tcnn_module.initial_params(seed)
        self.params = torch.nn.Parameter(initial_params, requires_grad=True)
        self.register_parameter(name="params", param=self.params)
        self.loss_scale = L.lib().tcnn_default_loss_scale(self.native_tcnn_module.param_precision())

    def forward(self, x):
        if not x.is_cuda:
            warnings.warn("input must be a CUDA tensor, but isn't. This indicates suboptimal performance.")
            x = x.cuda()
        batch_size = x.shape[0]
        g = _granularity()
        padded = (batch_size + g - 1) // g * g
        x_padded = x if batch_size == padded else torch.nn.functional.pad(x, [0, 0, 0, padded - batch_size])
        if x_padded.dtype != torch.float:
            x_padded = x_padded.to(torch.float)
        if not x_padded.is_contiguous():
            x_padded = x_padded.contiguous()
        params = self.params
        pdtype = self.native_tcnn_module._param_dtype
        if params.dtype != pdtype:
            params = params.to(pdtype)
        if not params.is_contiguous():
            params = params.contiguous()
        if _EXT is not None:
            output = _EXT.module_apply(self.native_tcnn_module.h, x_padded, params, float(self.loss_scale))
        else:
            output = _module_function.apply(self.native_tcnn_module, x_padded, params, self.loss_scale)
        if batch_size == padded and output.shape[1] == self.n_output_dims:
            return output
        return output[:batch_size, :self.n_output_dims]

    def __getstate__(self):
        """modules.py:194-199: pickle everything except the native module (a C-ABI handle)."""
        state = self.__dict__.copy()
        del state["native_tcnn_module"]
        return state

    def __setstate__(self, state):
        """modules.py:201-204: rebuild the native module from the stored configuration."""
        self.__dict__.update(state)
        self.native_tcnn_module = self._native_tcnn_module()

    def extra_repr(self):
        return (f"n_input_dims={self.n_input_dims}, n_output_dims={self.n_output_dims}, seed={self.seed}, "
                f"dtype={self.dtype}, hyperparams={self.native_tcnn_module.hyperparams()}")


class NetworkWithInputEncoding(Module):
    def __init__(self, n_input_dims, n_output_dims, encoding_config, network_config, seed=1337):
        if not _C.has_networks():
            raise RuntimeError("Cannot create `NetworkWithInputEncoding` because tiny-cuda-nn was not compiled with neural network support.")
        self.n_input_dims = n_input_dims
        self.n_output_dims = n_output_dims
        self.encoding_config = encoding_config
        self.network_config = network_config
        super().__init__(seed=seed)

    def _native_tcnn_module(self):
        return _NativeModule(L.lib().tcnn_create_network_with_input_encoding(
            self.n_input_dims, self.n_output_dims, json.dumps(self.encoding_config).encode(),
            json.dumps(self.network_config).encode()))


class Network(Module):
    def __init__(self, n_input_dims, n_output_dims, network_config, seed=1337):
        if not _C.has_networks():
            raise RuntimeError("Cannot create `Network` because tiny-cuda-nn was not compiled with neural network support.")
        self.n_input_dims = n_input_dims
        self.n_output_dims = n_output_dims
        self.network_config = network_config
        super().__init__(seed=seed)

    def _native_tcnn_module(self):
        return _NativeModule(L.lib().tcnn_create_network(self.n_input_dims, self.n_output_dims,
                                                          json.dumps(self.network_config).encode()))


class Encoding(Module):
    def __init__(self, n_input_dims, encoding_config, seed=1337, dtype=None):
        self.n_input_dims = n_input_dims
        self.encoding_config = encoding_config
        if dtype is None:
            self.precision = _C.preferred_precision()
        elif dtype == torch.float16:
            self.precision = PRECISION_FP16
        elif dtype == torch.float32:
            self.precision = PRECISION_FP32
        else:
            raise ValueError(f"Encoding only supports fp32 or fp16 precision, but got {dtype}")
        super().__init__(seed=seed)
        self.n_output_dims = self.native_tcnn_module.n_output_dims()

    def _native_tcnn_module(self):
        return _NativeModule(L.lib().tcnn_create_encoding(self.n_input_dims, json.dumps(self.encoding_config).encode(),
                                                           self.precision))
