"""ctypes binding of the in-tree HIP library dkg_amd/libdkg_amd.so (C ABI: include/dkg_amd.h).

The product path always runs the HIP kernels: there is no CPU fallback.  If the library is missing
or no GPU is visible, the calls below raise instead of silently computing something else.
"""
import ctypes
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DKG_AMD_LIB", os.path.join(HERE, "libdkg_amd.so"))

DKG_OK = 0
DKG_E_ARG = -1
DKG_E_DECODE = -2
DKG_E_DEVICE = -3
DKG_E_NOMEM = -4
REJECT, ACCEPT, SELF, SKIPPED, MISSING = 0, 1, 2, 3, 4
# per-party finalise status (dkg_finalise_parties)
FIN_OK, FIN_R2_ERROR, FIN_R4_ERROR, FIN_PHASE4_ERROR, FIN_INSUFFICIENT, FIN_PANIC = 0, 1, 2, 3, 4, 5

_lib = None


class DkgError(RuntimeError):
    def __init__(self, code, msg=""):
        self.code = code
        names = {DKG_E_ARG: "DKG_E_ARG", DKG_E_DECODE: "DKG_E_DECODE", DKG_E_DEVICE: "DKG_E_DEVICE",
                 DKG_E_NOMEM: "DKG_E_NOMEM"}
        super().__init__(f"{names.get(code, code)}: {msg}")


class CeremonyOut(ctypes.Structure):
    _fields_ = [
        ("E", ctypes.c_void_p), ("A", ctypes.c_void_p),
        ("s", ctypes.c_void_p), ("s_prime", ctypes.c_void_p),
        ("dec2", ctypes.c_void_p), ("dec4", ctypes.c_void_p),
        ("qualified", ctypes.c_void_p), ("r2_error", ctypes.c_void_p), ("r4_error", ctypes.c_void_p),
        ("complaints2", ctypes.c_void_p), ("reconstruct", ctypes.c_void_p),
        ("final_share", ctypes.c_void_p), ("public_share", ctypes.c_void_p),
        ("mpk", ctypes.c_uint8 * 32),
        ("n_qualified", ctypes.c_int32), ("phase4_error", ctypes.c_int32),
        ("ms_round1", ctypes.c_double), ("ms_round2", ctypes.c_double), ("ms_round3", ctypes.c_double),
        ("ms_round4", ctypes.c_double), ("ms_finalise", ctypes.c_double), ("ms_total", ctypes.c_double),
    ]


class ShardOutcome(ctypes.Structure):
    _fields_ = [
        ("qualified", ctypes.c_void_p), ("complaints2", ctypes.c_void_p), ("r2_error", ctypes.c_void_p),
        ("reconstruct", ctypes.c_void_p), ("r4_error", ctypes.c_void_p),
        ("n_qualified", ctypes.c_int32), ("phase4_error", ctypes.c_int32),
    ]


class BatchOut(ctypes.Structure):
    _fields_ = [
        ("mpk", ctypes.c_void_p), ("n_qualified", ctypes.c_void_p), ("phase4_error", ctypes.c_void_p),
        ("qualified", ctypes.c_void_p),
        ("r2_error", ctypes.c_void_p), ("r4_error", ctypes.c_void_p), ("complaints2", ctypes.c_void_p),
        ("reconstruct", ctypes.c_void_p), ("final_share", ctypes.c_void_p), ("public_share", ctypes.c_void_p),
        ("dec2", ctypes.c_void_p), ("dec4", ctypes.c_void_p),
        ("ms_round1", ctypes.c_double), ("ms_checks", ctypes.c_double), ("ms_round3", ctypes.c_double),
        ("ms_finalise", ctypes.c_double), ("ms_total", ctypes.c_double),
    ]


def lib():
    """Load libdkg_amd.so (raises if it is absent: the HIP path is mandatory)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} is missing: build it with `make -C dkg_amd` or __graft_entry__.build()")
    # When torch shares the process, its HIP runtime must be the one the dynamic loader binds
    # first: loading libdkg_amd.so (linked against /opt/rocm's libamdhip64) before torch leaves
    # torch.cuda without a device.  Import torch first whenever it is importable; a torch install
    # that fails to import for any reason (its ROCm libraries included) must not stop the library
    # from loading for callers that never use torch (DKG_NO_TORCH_PREIMPORT=1 skips the attempt).
    if "torch" not in sys.modules and not os.environ.get("DKG_NO_TORCH_PREIMPORT"):
        try:
            import torch  # noqa: F401
        except Exception:  # noqa: BLE001 -- ImportError, OSError, RuntimeError from a broken install
            pass
    L = ctypes.CDLL(LIB_PATH)
    sz, p, u8p = ctypes.c_size_t, ctypes.c_void_p, ctypes.c_char_p
    L.dkg_ctx_create.argtypes = [ctypes.c_int, ctypes.POINTER(p)]
    L.dkg_ctx_destroy.argtypes = [p]
    L.dkg_ctx_destroy.restype = None
    L.dkg_ctx_last_error.argtypes = [p]
    L.dkg_ctx_last_error.restype = ctypes.c_char_p
    L.dkg_device_count.argtypes = []
    L.dkg_ctx_set_streams.argtypes = [p, ctypes.c_int]
    L.dkg_ctx_set_overlap.argtypes = [p, ctypes.c_int]
    L.dkg_ctx_set_verify_mode.argtypes = [p, ctypes.c_int]
    L.dkg_ctx_fallback_rows.argtypes = [p]
    L.dkg_ctx_fallback_rows.restype = sz
    L.dkg_ctx_set_split.argtypes = [p, ctypes.c_int]
    L.dkg_ctx_set_stepping.argtypes = [p, ctypes.c_int]
    L.dkg_ctx_set_field_mode.argtypes = [p, ctypes.c_int]
    L.dkg_ctx_set_binomial.argtypes = [p, ctypes.c_int]
    L.dkg_ctx_set_check.argtypes = [p, ctypes.c_int]
    L.dkg_ctx_last_split.argtypes = [p]
    L.dkg_ctx_last_split_len.argtypes = [p]
    L.dkg_ctx_last_split_len.restype = sz
    L.dkg_split_model_ms.argtypes = [sz, sz, sz, ctypes.c_int]
    L.dkg_split_model_ms.restype = ctypes.c_double
    L.dkg_split_len.argtypes = [sz, sz, sz, ctypes.c_int]
    L.dkg_split_len.restype = sz
    L.dkg_ctx_set_combine.argtypes = [p, ctypes.c_int]
    L.dkg_ctx_last_combine.argtypes = [p]
    L.dkg_ctx_last_binomial.argtypes = [p]
    L.dkg_ctx_set_addends.argtypes = [p, ctypes.c_int]
    L.dkg_ctx_set_stepping_formula.argtypes = [p, ctypes.c_int]
    L.dkg_ctx_stepping_redos.argtypes = [p]
    L.dkg_ctx_stepping_redos.restype = ctypes.c_longlong
    L.dkg_ctx_binomial_reruns.argtypes = [p]
    L.dkg_ctx_clock_probe.argtypes = [p, ctypes.c_uint, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]
    L.dkg_device_pci_bus_id.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_int]
    L.dkg_split_multipliers.argtypes = [sz, sz, ctypes.c_int, p, p]
    L.dkg_ctx_phase_ms.argtypes = [p, ctypes.c_char_p]
    L.dkg_ctx_phase_ms.restype = ctypes.c_double
    L.dkg_env_check.argtypes = [sz, sz]
    L.dkg_env_init.argtypes = [p, sz, sz, u8p, sz, p]
    L.dkg_msm_batch.argtypes = [p, sz, sz, u8p, u8p, p]
    L.dkg_fixed_base_batch.argtypes = [p, p, sz, u8p, p]
    L.dkg_poly_eval_batch.argtypes = [p, sz, sz, u8p, sz, p, p]
    L.dkg_points_valid_batch.argtypes = [p, sz, u8p, p]
    L.dkg_share_gen.argtypes = [p, sz, sz, sz, u8p, u8p, p, p, p, p]
    L.dkg_verify_pairs.argtypes = [p, sz, sz, ctypes.c_int, sz, sz, u8p, u8p, p, p]
    L.dkg_verify_receiver.argtypes = [p, sz, sz, ctypes.c_int, sz, u8p, u8p, p, p]
    L.dkg_ceremony_run.argtypes = [p, sz, sz, u8p, u8p, ctypes.POINTER(CeremonyOut)]
    L.dkg_ceremony_verify.argtypes = [p, sz, sz, u8p, u8p, u8p, u8p, ctypes.POINTER(CeremonyOut)]
    L.dkg_ceremony_verify_fetched.argtypes = [p, sz, sz, u8p, u8p, u8p, u8p, u8p, u8p, ctypes.POINTER(CeremonyOut)]
    L.dkg_ceremony_run_device.argtypes = [p, sz, sz, p, p, ctypes.POINTER(CeremonyOut)]
    L.dkg_ceremony_shard_device.argtypes = [p, sz, sz, sz, sz, p, p, p, p, p, p, ctypes.POINTER(ctypes.c_double)]
    L.dkg_ceremony_shard_verify_device.argtypes = [p, sz, sz, sz, sz, p, p, p, p, p, p, p, p,
                                                    ctypes.POINTER(ctypes.c_double)]
    L.dkg_ceremony_batch_device.argtypes = [p, sz, sz, sz, p, p, ctypes.POINTER(BatchOut)]
    L.dkg_ceremony_batch_verify.argtypes = [p, sz, sz, sz, u8p, u8p, u8p, u8p, ctypes.POINTER(BatchOut)]
    L.dkg_dealer_coeffs_device.argtypes = [p, u8p, ctypes.c_uint32, sz, sz, sz, sz, p, p]
    L.dkg_member_keys.argtypes = [p, u8p, ctypes.c_uint32, sz, p, p]
    L.dkg_enc_randomness.argtypes = [u8p, ctypes.c_uint32, sz, sz, sz, sz, p]
    L.dkg_enc_randomness_device.argtypes = [p, u8p, ctypes.c_uint32, sz, sz, sz, sz, sz, p]
    L.dkg_encrypt_shares.argtypes = [p, sz, sz, u8p, u8p, u8p, u8p, p, p]
    L.dkg_decrypt_shares.argtypes = [p, sz, sz, u8p, u8p, u8p, p, p, p]
    L.dkg_ceremony_run_full_device.argtypes = [p, sz, sz, p, p, p, u8p, u8p, ctypes.POINTER(CeremonyOut)]
    L.dkg_ceremony_verify_full.argtypes = [p, sz, sz, u8p, u8p, u8p, u8p, u8p, ctypes.POINTER(CeremonyOut)]
    L.dkg_misbehaviour_prove.argtypes = [p, sz, u8p, u8p, u8p, p]
    L.dkg_complaint1_verify.argtypes = [p, sz, sz, p, u8p, u8p, u8p, u8p, p]
    L.dkg_complaint3_verify.argtypes = [p, sz, sz, p, u8p, u8p, u8p, u8p, p]
    L.dkg_dealer_coeffs.argtypes = [u8p, ctypes.c_uint32, sz, sz, sz, p, p]
    L.dkg_scalar_sum_device.argtypes = [p, sz, sz, p, p, p]
    L.dkg_point_sum_device.argtypes = [p, sz, p, p, p]
    L.dkg_share_gen_device.argtypes = [p, sz, sz, sz, p, p, p, p, p, p]
    L.dkg_ceremony_shard_recon_device.argtypes = [p, sz, sz, sz, sz, u8p, u8p, u8p, u8p, p, p,
                                                  ctypes.POINTER(ctypes.c_int32)]
    L.dkg_finalise_parties.argtypes = [p, sz, sz, u8p, u8p, u8p, u8p, u8p, u8p, u8p, p, p, p]
    L.dkg_shard_range.argtypes = [sz, sz, sz, ctypes.POINTER(sz), ctypes.POINTER(sz)]
    L.dkg_shard_range.restype = None
    L.dkg_shard_rows.argtypes = [sz, sz]
    L.dkg_shard_rows.restype = sz
    L.dkg_shard_combine_device.argtypes = [p, sz, sz, sz, p, p, p, p, ctypes.POINTER(ShardOutcome)]
    L.dkg_shard_combine_packed_device.argtypes = [p, sz, sz, sz, p, p, p, p, ctypes.POINTER(ShardOutcome)]
    L.dkg_fixed_base_windows.argtypes = []
    L.dkg_key_comb_windows.argtypes = []
    L.dkg_packed_row_words.argtypes = [sz]
    L.dkg_packed_row_words.restype = sz
    L.dkg_decisions_pack_device.argtypes = [p, sz, sz, sz, sz, p, p]
    L.dkg_shard_finalise_device.argtypes = [p, sz, sz, sz, p, p, u8p, ctypes.c_int, p, p, p]
    L.dkg_multi_create.argtypes = [ctypes.POINTER(ctypes.c_int), ctypes.c_int, ctypes.POINTER(p)]
    L.dkg_multi_destroy.argtypes = [p]
    L.dkg_multi_destroy.restype = None
    L.dkg_multi_size.argtypes = [p]
    L.dkg_multi_ctx.argtypes = [p, ctypes.c_int]
    L.dkg_multi_ctx.restype = p
    L.dkg_multi_last_error.argtypes = [p]
    L.dkg_multi_last_error.restype = ctypes.c_char_p
    L.dkg_multi_phase_ms.argtypes = [p, ctypes.c_char_p]
    L.dkg_multi_phase_ms.restype = ctypes.c_double
    L.dkg_multi_env_init.argtypes = [p, sz, sz, u8p, sz, p]
    L.dkg_multi_ceremony_run.argtypes = [p, sz, sz, u8p, u8p, ctypes.POINTER(CeremonyOut)]
    L.dkg_multi_ceremony_run_device.argtypes = [p, sz, sz, ctypes.POINTER(p), ctypes.POINTER(p),
                                                ctypes.POINTER(CeremonyOut)]
    L.dkg_multi_ceremony_verify.argtypes = [p, sz, sz, u8p, u8p, u8p, u8p, ctypes.POINTER(CeremonyOut)]
    _lib = L
    return L


EXPORTED = [
    "dkg_ctx_create", "dkg_ctx_destroy", "dkg_ctx_last_error", "dkg_ctx_phase_ms", "dkg_ctx_set_streams", "dkg_ctx_set_overlap",
    "dkg_device_count", "dkg_env_init",
    "dkg_env_check", "dkg_msm_batch", "dkg_fixed_base_batch", "dkg_poly_eval_batch",
    "dkg_points_valid_batch", "dkg_share_gen", "dkg_verify_pairs", "dkg_verify_receiver",
    "dkg_ctx_set_split", "dkg_ctx_set_stepping", "dkg_ctx_set_field_mode", "dkg_ctx_set_binomial", "dkg_ctx_set_check", "dkg_ctx_last_split", "dkg_ctx_last_split_len", "dkg_ctx_set_verify_mode", "dkg_ctx_fallback_rows", "dkg_split_model_ms", "dkg_split_len",
    "dkg_ctx_set_combine", "dkg_ctx_last_combine", "dkg_ctx_last_binomial", "dkg_ctx_set_addends", "dkg_ctx_set_stepping_formula", "dkg_ctx_stepping_redos", "dkg_ctx_binomial_reruns", "dkg_split_multipliers",
    "dkg_ctx_clock_probe", "dkg_device_pci_bus_id",
    "dkg_ceremony_run", "dkg_ceremony_verify", "dkg_ceremony_verify_fetched", "dkg_ceremony_run_device", "dkg_ceremony_shard_device",
    "dkg_ceremony_shard_verify_device",
    "dkg_ceremony_batch_device", "dkg_ceremony_batch_verify", "dkg_member_keys", "dkg_enc_randomness",
    "dkg_enc_randomness_device", "dkg_encrypt_shares", "dkg_decrypt_shares", "dkg_ceremony_run_full_device",
    "dkg_ceremony_verify_full", "dkg_misbehaviour_prove", "dkg_complaint1_verify", "dkg_complaint3_verify", "dkg_dealer_coeffs", "dkg_dealer_coeffs_device",
    "dkg_scalar_sum_device", "dkg_point_sum_device", "dkg_ceremony_shard_recon_device", "dkg_finalise_parties",
    "dkg_share_gen_device", "dkg_shard_range", "dkg_shard_rows", "dkg_shard_combine_device",
    "dkg_shard_combine_packed_device", "dkg_packed_row_words", "dkg_fixed_base_windows", "dkg_key_comb_windows", "dkg_decisions_pack_device",
    "dkg_shard_finalise_device", "dkg_multi_create", "dkg_multi_destroy", "dkg_multi_size", "dkg_multi_ctx",
    "dkg_multi_last_error", "dkg_multi_phase_ms", "dkg_multi_env_init", "dkg_multi_ceremony_run",
    "dkg_multi_ceremony_run_device", "dkg_multi_ceremony_verify",
]
