"""ctypes binding of the C-ABI (include/tcnn_mi355x.h) exported by lib/libtcnn_mi355x.so.

The HIP library is the only compute path: if it is missing this module raises immediately (there is
no CPU / eager-PyTorch fallback).
"""
import ctypes
import os

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# TCNN_LIB_PATH: another build of the same library (A/B timing of two builds in one job)
LIB_PATH = os.environ.get("TCNN_LIB_PATH") or os.path.join(_PKG, "lib", "libtcnn_mi355x.so")

_lib = None

c_void_p, c_float, c_int, c_uint32, c_uint64, c_char_p = (
    ctypes.c_void_p, ctypes.c_float, ctypes.c_int, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_char_p)

# void (*)(int severity, const char* message, void* user) -- tcnn_set_log_callback
LOG_CALLBACK = ctypes.CFUNCTYPE(None, c_int, c_char_p, c_void_p)

_SIGS = {
    "tcnn_last_error": (c_char_p, []),
    "tcnn_version": (c_char_p, []),
    "tcnn_batch_size_granularity": (c_uint32, []),
    "tcnn_cuda_device": (c_int, []),
    "tcnn_set_cuda_device": (c_int, [c_int]),
    "tcnn_free_temporary_memory": (None, []),
    "tcnn_has_networks": (c_int, []),
    "tcnn_default_loss_scale": (c_float, [c_int]),
    "tcnn_preferred_precision": (c_int, []),
    "tcnn_set_log_callback": (None, [LOG_CALLBACK, c_void_p]),
    "tcnn_generate_random_uniform": (c_int, [c_void_p, c_void_p, c_void_p, c_uint64, c_void_p, c_float, c_float]),
    "tcnn_generate_random_logistic": (c_int, [c_void_p, c_void_p, c_void_p, c_uint64, c_void_p, c_float, c_float]),
    "tcnn_create_network_with_input_encoding": (c_void_p, [c_uint32, c_uint32, c_char_p, c_char_p]),
    "tcnn_create_network": (c_void_p, [c_uint32, c_uint32, c_char_p]),
    "tcnn_create_encoding": (c_void_p, [c_uint32, c_char_p, c_int]),
    "tcnn_module_destroy": (None, [c_void_p]),
    "tcnn_module_inference": (c_int, [c_void_p, c_void_p, c_uint32, c_void_p, c_void_p, c_void_p]),
    "tcnn_module_forward": (c_void_p, [c_void_p, c_void_p, c_uint32, c_void_p, c_void_p, c_void_p, c_int]),
    "tcnn_module_backward": (c_int, [c_void_p, c_void_p, c_void_p, c_uint32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "tcnn_module_backward_scaled": (c_int, [c_void_p, c_void_p, c_void_p, c_uint32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_float, c_int]),
    "tcnn_module_backward_backward_input": (c_int, [c_void_p, c_void_p, c_void_p, c_uint32] + [c_void_p] * 7),
    "tcnn_context_destroy": (None, [c_void_p]),
    "tcnn_module_set_max_level": (c_int, [c_void_p, c_float]),
    "tcnn_module_max_level": (c_float, [c_void_p]),
    "tcnn_module_set_max_level_gpu": (c_int, [c_void_p, c_void_p]),
    "tcnn_trainer_set_max_level": (c_int, [c_void_p, c_float]),
    "tcnn_module_n_input_dims": (c_uint32, [c_void_p]),
    "tcnn_module_n_output_dims": (c_uint32, [c_void_p]),
    "tcnn_module_n_params": (c_uint64, [c_void_p]),
    "tcnn_module_param_precision": (c_int, [c_void_p]),
    "tcnn_module_output_precision": (c_int, [c_void_p]),
    "tcnn_module_initialize_params": (c_int, [c_void_p, c_uint64, c_void_p, c_float]),
    "tcnn_module_hyperparams": (c_char_p, [c_void_p]),
    "tcnn_module_name": (c_char_p, [c_void_p]),
    "tcnn_trainer_create": (c_void_p, [c_uint32, c_uint32, c_char_p, c_uint32]),
    "tcnn_trainer_destroy": (None, [c_void_p]),
    "tcnn_trainer_training_step": (c_int, [c_void_p, c_void_p, c_uint32, c_void_p, c_void_p, c_int]),
    "tcnn_trainer_optimizer_step": (c_int, [c_void_p, c_void_p]),
    "tcnn_trainer_forward": (c_void_p, [c_void_p, c_void_p, c_uint32, c_void_p, c_void_p, c_void_p, c_void_p, c_int]),
    "tcnn_trainer_forward_perturbed": (c_void_p, [c_void_p, c_void_p, c_uint32, c_void_p, c_void_p, c_void_p, c_void_p, c_int]),
    "tcnn_trainer_backward": (c_int, [c_void_p, c_void_p, c_void_p, c_uint32, c_void_p, c_void_p, c_int]),
    "tcnn_trainer_context_loss": (c_float, [c_void_p, c_void_p, c_void_p]),
    "tcnn_trainer_context_output": (c_void_p, [c_void_p]),
    "tcnn_trainer_context_doutput": (c_void_p, [c_void_p]),
    "tcnn_trainer_context_destroy": (None, [c_void_p]),
    "tcnn_trainer_padded_output_width": (c_uint32, [c_void_p]),
    "tcnn_workspace_allocate": (c_void_p, [c_void_p, c_uint64]),
    "tcnn_workspace_free": (c_int, [c_void_p, c_void_p]),
    "tcnn_free_workspace_arena": (c_int, [c_void_p]),
    "tcnn_workspace_arena_info": (c_int, [c_void_p, c_void_p, c_void_p]),
    "tcnn_trainer_optimizer_step_range": (c_int, [c_void_p, c_void_p, c_uint64, c_uint64]),
    "tcnn_trainer_training_step_part": (c_int, [c_void_p, c_void_p, c_uint32, c_void_p, c_void_p, c_int]),
    "tcnn_trainer_loss": (c_float, [c_void_p, c_void_p]),
    "tcnn_trainer_loss_device": (c_void_p, [c_void_p]),
    "tcnn_trainer_inference": (c_int, [c_void_p, c_void_p, c_uint32, c_void_p, c_void_p]),
    "tcnn_trainer_n_params": (c_uint64, [c_void_p]),
    "tcnn_trainer_n_network_params": (c_uint64, [c_void_p]),
    "tcnn_trainer_params_fp32": (c_void_p, [c_void_p]),
    "tcnn_trainer_params": (c_void_p, [c_void_p]),
    "tcnn_trainer_param_gradients": (c_void_p, [c_void_p]),
    "tcnn_trainer_gradients_fp32": (c_void_p, [c_void_p]),
    "tcnn_trainer_set_gradient_scale": (c_int, [c_void_p, c_float]),
    "tcnn_trainer_set_loss_scale": (c_int, [c_void_p, c_float]),
    "tcnn_trainer_set_graph": (c_int, [c_void_p, c_int]),
    "tcnn_trainer_graph_stats": (c_int, [c_void_p, c_void_p, c_void_p]),
    "tcnn_trainer_set_params_full_precision": (c_int, [c_void_p, c_void_p, c_uint64]),
    "tcnn_trainer_optimizer_step_count": (c_uint32, [c_void_p]),
    "tcnn_trainer_update_hyperparams": (c_int, [c_void_p, c_char_p]),
    "tcnn_trainer_hyperparams": (c_char_p, [c_void_p]),
    "tcnn_trainer_initialize_params": (c_int, [c_void_p, c_uint32]),
    "tcnn_trainer_initialize_params_rng": (c_int, [c_void_p, c_void_p, c_uint64]),
    "tcnn_trainer_engine": (c_char_p, [c_void_p]),
    "tcnn_trainer_optimizer_state": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p]),
    "tcnn_dp_unique_id": (c_int, [c_void_p]),
    "tcnn_dp_comm_create": (c_void_p, [c_void_p, c_int, c_int]),
    "tcnn_dp_comm_destroy": (None, [c_void_p]),
    "tcnn_trainer_set_dp": (c_int, [c_void_p, c_void_p, c_int]),
    "tcnn_trainer_dp_gather_state": (c_int, [c_void_p, c_void_p]),
    "tcnn_dp_peer_blob_bytes": (c_uint64, []),
    "tcnn_trainer_dp_peer_export": (c_int, [c_void_p, c_int, c_int, c_void_p]),
    "tcnn_trainer_dp_peer_attach": (c_int, [c_void_p, c_void_p]),
    "tcnn_trainer_dp_peer_detach": (c_int, [c_void_p]),
    "tcnn_trainer_dp_peer_abandon": (c_int, [c_void_p]),
    "tcnn_trainer_dp_peer_set_timeout": (c_int, [c_void_p, ctypes.c_double]),
    "tcnn_trainer_inference_engine": (c_char_p, [c_void_p]),
    "tcnn_module_engine": (c_char_p, [c_void_p]),
    "tcnn_module_inference_engine": (c_char_p, [c_void_p]),
    "tcnn_trainer_profile_begin": (c_int, [c_void_p]),
    "tcnn_trainer_profile_begin_sampled": (c_int, [c_void_p, c_uint32]),
    "tcnn_trainer_serialize": (c_int, [c_void_p, c_int, c_void_p, c_uint64, c_void_p]),
    "tcnn_trainer_serialize_json": (c_int, [c_void_p, c_int, c_void_p, c_uint64, c_void_p]),
    "tcnn_trainer_deserialize": (c_int, [c_void_p, c_void_p, c_uint64]),
    "tcnn_trainer_profile_end": (c_int, [c_void_p, c_void_p, c_uint32, c_void_p]),
}

# test-only diagnostics (neuralbtf-tiny-cuda-nn_amd/csrc/debug_api.h, not the product C-ABI header)
_DEBUG_SIGS = {
    "tcnn_debug_probe": (c_int, [c_void_p, c_void_p, c_void_p]),
    "tcnn_debug_fused_phase_cycles": (c_int, [c_void_p, c_void_p, c_uint32, c_void_p, c_void_p, c_void_p]),
    "tcnn_debug_hfma": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_uint32]),
    "tcnn_debug_peer_loopback": (c_int, [c_void_p, c_int]),
}


class TcnnError(RuntimeError):
    pass


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"tinycudann (MI355X): HIP library not built: {LIB_PATH} is missing. "
                "Run `make -C neuralbtf-tiny-cuda-nn_amd` or __graft_entry__.build().")
        _lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in list(_SIGS.items()) + list(_DEBUG_SIGS.items()):
            f = getattr(_lib, name)
            f.restype = res
            f.argtypes = args
    return _lib


def exported_symbols():
    return list(_SIGS.keys())


def debug_symbols():
    return list(_DEBUG_SIGS.keys())


def check(rc):
    if rc != 0:
        raise TcnnError(lib().tcnn_last_error().decode())


def check_ptr(p):
    if not p:
        raise TcnnError(lib().tcnn_last_error().decode())
    return p
