"""create_from_config() / Trainer front-end (reference include/tiny-cuda-nn/config.h:46-63,
trainer.h:47-361) over the C-ABI tcnn_trainer_* entry points. Inputs/outputs are torch CUDA tensors
(device memory); the stream is torch's current stream."""
import ctypes
import json

from tinycudann import _lib as L


def _stream(stream=None):
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


class Trainer:
    def __init__(self, n_input_dims, n_output_dims, config, seed=1337):
        self.n_input_dims = n_input_dims
        self.n_output_dims = n_output_dims
        self.config = config
        self.h = L.check_ptr(L.lib().tcnn_trainer_create(n_input_dims, n_output_dims, json.dumps(config).encode(), seed))
        self.n_params = L.lib().tcnn_trainer_n_params(self.h)
        self.n_network_params = L.lib().tcnn_trainer_n_network_params(self.h)

    def __del__(self):
        try:
            L.lib().tcnn_trainer_destroy(self.h)
        except Exception:
            pass

    @property
    def engine(self):
        return L.lib().tcnn_trainer_engine(self.h).decode()

    @property
    def inference_engine(self):
        return L.lib().tcnn_trainer_inference_engine(self.h).decode()

    def training_step(self, input, target, run_optimizer=True, stream=None):
        """input: float32 [B, n_in] CUDA, target float32 [B, n_out] CUDA (contiguous)."""
        assert input.is_contiguous() and target.is_contiguous()
        L.check(L.lib().tcnn_trainer_training_step(self.h, _stream(stream), input.shape[0], ctypes.c_void_p(input.data_ptr()),
                                                   ctypes.c_void_p(target.data_ptr()), int(run_optimizer)))

    def training_step_part(self, input, target, part, stream=None):
        """Data-parallel split of training_step(run_optimizer=False): part 0 leaves the network
        gradients final (gradients_fp32()[:n_network_params]), part 1 runs the grid backward."""
        assert input.is_contiguous() and target.is_contiguous()
        L.check(L.lib().tcnn_trainer_training_step_part(self.h, _stream(stream), input.shape[0], ctypes.c_void_p(input.data_ptr()),
                                                        ctypes.c_void_p(target.data_ptr()), int(part)))

    def optimizer_step(self, stream=None):
        L.check(L.lib().tcnn_trainer_optimizer_step(self.h, _stream(stream)))

    @property
    def padded_output_width(self):
        return L.lib().tcnn_trainer_padded_output_width(self.h)

    def forward(self, input, target=None, data_pdf=None, external_dL_dy=None, prepare_input_gradients=False, stream=None):
        """Trainer::forward (trainer.h:97-144): network output + loss on target (optionally weighted by
        data_pdf float32 [B, n_out]), or the caller's loss-scaled dL/dy (float16 [B, padded_output_width]).
        Returns a ForwardContext for backward() / its loss()."""
        for t in (input, target, data_pdf, external_dL_dy):
            assert t is None or t.is_contiguous()
        ptr = lambda t: ctypes.c_void_p(t.data_ptr() if t is not None else 0)
        h = L.lib().tcnn_trainer_forward(self.h, _stream(stream), input.shape[0], ptr(input), ptr(target), ptr(data_pdf),
                                         ptr(external_dL_dy), int(prepare_input_gradients))
        return ForwardContext(self, L.check_ptr(h), input.shape[0], (input, target, data_pdf, external_dL_dy))

    def backward(self, ctx, input, dL_dinput=None, accumulate=False, stream=None, gradient_mode=None):
        """Trainer::backward (trainer.h:146-153): parameter gradients into gradients_fp32()
        (Overwrite, or Accumulate with accumulate=True) and optionally dL/dinput (float32 [B, n_in]).
        gradient_mode ("overwrite" | "accumulate" | "ignore", GradientMode, common.h) overrides
        `accumulate`; "ignore" leaves the parameter gradients untouched and only writes dL/dinput."""
        assert ctx.trainer is self
        modes = {"overwrite": 0, "accumulate": 1, "ignore": 2}
        mode = modes[gradient_mode.lower()] if gradient_mode is not None else int(bool(accumulate))
        L.check(L.lib().tcnn_trainer_backward(self.h, _stream(stream), ctx.h, input.shape[0], ctypes.c_void_p(input.data_ptr()),
                                              ctypes.c_void_p(dL_dinput.data_ptr() if dL_dinput is not None else 0),
                                              mode))

    def optimizer_step_range(self, begin, end, stream=None):
        """Adam on parameters [begin, end) only (one optimizer step; data-parallel sharded optimizer)."""
        L.check(L.lib().tcnn_trainer_optimizer_step_range(self.h, _stream(stream), int(begin), int(end)))

    def loss(self, stream=None):
        v = L.lib().tcnn_trainer_loss(self.h, _stream(stream))
        if v < 0:
            raise L.TcnnError(L.lib().tcnn_last_error().decode())
        return v

    def inference(self, input, stream=None):
        import torch
        out = torch.empty(input.shape[0], self.n_output_dims, dtype=torch.float32, device=input.device)
        L.check(L.lib().tcnn_trainer_inference(self.h, _stream(stream), input.shape[0], ctypes.c_void_p(input.data_ptr()),
                                               ctypes.c_void_p(out.data_ptr())))
        return out

    def set_graph(self, on=True):
        """Replay the training step as a hipGraph while its inputs are unchanged (the reference
        Trainer's CUDA graph, trainer.h:163-190); bit-identical to the eager step."""
        L.check(L.lib().tcnn_trainer_set_graph(self.h, int(bool(on))))

    def graph_stats(self):
        """(captures, replays) of the training-step graph."""
        c, r = ctypes.c_uint64(0), ctypes.c_uint64(0)
        L.check(L.lib().tcnn_trainer_graph_stats(self.h, ctypes.byref(c), ctypes.byref(r)))
        return c.value, r.value

    def set_gradient_scale(self, s):
        L.check(L.lib().tcnn_trainer_set_gradient_scale(self.h, float(s)))

    def set_loss_scale(self, s):
        """the loss scale of training_step / forward / optimizer_step (the reference's loss_scale
        argument, trainer.h:97-160; default 128)"""
        L.check(L.lib().tcnn_trainer_set_loss_scale(self.h, float(s)))

    def set_params_full_precision(self, host_params):
        import numpy as np
        a = np.ascontiguousarray(host_params, dtype=np.float32)
        L.check(L.lib().tcnn_trainer_set_params_full_precision(self.h, a.ctypes.data_as(ctypes.c_void_p), a.size))

    def serialize(self, optimizer=False):
        """Trainer::serialize as the reference's msgpack snapshot bytes (trainer.h:275-288)."""
        if optimizer and getattr(self, "_dp_state_partial", False):
            raise L.TcnnError("serialize(optimizer=True): the sharded data-parallel optimizer state is current only on each "
                              "rank's shard; call DataParallelTrainer.gather_state() first")
        n = ctypes.c_uint64(0)
        L.check(L.lib().tcnn_trainer_serialize(self.h, int(optimizer), None, 0, ctypes.byref(n)))
        buf = ctypes.create_string_buffer(n.value)
        L.check(L.lib().tcnn_trainer_serialize(self.h, int(optimizer), buf, n.value, ctypes.byref(n)))
        return buf.raw[:n.value]

    def deserialize(self, data):
        """Trainer::deserialize from msgpack snapshot bytes (trainer.h:290-315)."""
        b = bytes(data)
        L.check(L.lib().tcnn_trainer_deserialize(self.h, b, len(b)))

    def save_snapshot(self, path, optimizer=True):
        with open(path, "wb") as f:
            f.write(self.serialize(optimizer))

    def load_snapshot(self, path):
        with open(path, "rb") as f:
            self.deserialize(f.read())

    @property
    def optimizer_step_count(self):
        return L.lib().tcnn_trainer_optimizer_step_count(self.h)

    def _view(self, ptr, n, dtype):
        """torch view of a trainer-owned device buffer (via __cuda_array_interface__)."""
        import torch
        typestr = {torch.float32: "<f4", torch.float16: "<f2", torch.int32: "<i4"}[dtype]

        class _Iface:
            __cuda_array_interface__ = {"shape": (n,), "typestr": typestr, "data": (ptr, False), "version": 2}

        return torch.as_tensor(_Iface(), device="cuda")

    def params_fp32(self):
        import torch
        return self._view(L.lib().tcnn_trainer_params_fp32(self.h), self.n_params, torch.float32)

    def params(self):
        import torch
        return self._view(L.lib().tcnn_trainer_params(self.h), self.n_params, torch.float16)

    def param_gradients(self):
        import torch
        return self._view(L.lib().tcnn_trainer_param_gradients(self.h), self.n_params, torch.float16)

    def gradients_fp32(self):
        import torch
        return self._view(L.lib().tcnn_trainer_gradients_fp32(self.h), self.n_params, torch.float32)

    def optimizer_state(self):
        """(first moments fp32, second moments fp32, per-parameter step counts int32) views (adam.h:128-148)"""
        import torch
        m1, m2, st = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
        L.check(L.lib().tcnn_trainer_optimizer_state(self.h, ctypes.byref(m1), ctypes.byref(m2), ctypes.byref(st)))
        return (self._view(m1.value, self.n_params, torch.float32), self._view(m2.value, self.n_params, torch.float32),
                self._view(st.value, self.n_params, torch.int32))

    def set_dp(self, comm, sharded=False):
        """Attach an engine data-parallel communicator (tinycudann.parallel.EngineComm; None detaches):
        every training_step(run_optimizer=True) then sums the gradients across the ranks inside the
        step (tcnn_trainer_set_dp)."""
        L.check(L.lib().tcnn_trainer_set_dp(self.h, comm.h if comm is not None else None, int(bool(sharded))))
        self._dp_comm = comm  # the communicator must outlive the attachment

    def dp_gather_state(self, stream=None):
        """All-gather the sharded optimizer state (fp32 masters, Adam moments, steps) of an attached
        engine communicator (tcnn_trainer_dp_gather_state), e.g. before serialize(optimizer=True)."""
        L.check(L.lib().tcnn_trainer_dp_gather_state(self.h, _stream(stream)))


def create_from_config(n_input_dims, n_output_dims, config, seed=1337):
    """TrainableModel equivalent: returns the Trainer (which owns loss, optimizer and network)."""
    return Trainer(n_input_dims, n_output_dims, config, seed)


class ForwardContext:
    """Trainer::ForwardContext (trainer.h:89-95): owns the engine's context (output, dL/doutput, loss)."""

    def __init__(self, trainer, h, n, keepalive):
        self.trainer, self.h, self.n = trainer, h, n
        self._keep = keepalive  # the caller's tensors the queued kernels read

    def __del__(self):
        try:
            L.lib().tcnn_trainer_context_destroy(self.h)
        except Exception:
            pass

    def _view(self, ptr):
        import torch

        class _Dev:  # zero-copy view of engine memory (__cuda_array_interface__), cloned below
            pass

        w = self.trainer.padded_output_width
        d = _Dev()
        d.__cuda_array_interface__ = {"shape": (self.n, w), "typestr": "<f2", "data": (int(ptr), False), "version": 2}
        return torch.as_tensor(d, device="cuda").clone()

    @property
    def output(self):
        """fp16 [B, padded_output_width] copy of the network output."""
        return self._view(L.lib().tcnn_trainer_context_output(self.h))

    @property
    def dL_doutput(self):
        return self._view(L.lib().tcnn_trainer_context_doutput(self.h))

    def loss(self, stream=None):
        v = L.lib().tcnn_trainer_context_loss(self.trainer.h, _stream(stream), self.h)
        if v < 0:
            raise L.TcnnError(L.lib().tcnn_last_error().decode())
        return v
