"""ctypes signatures of libdtf_runtime.so (csrc/runtime/*.cc)."""
import ctypes

P, I, U32, I64, U64, D, F, S = (ctypes.c_void_p, ctypes.c_int, ctypes.c_uint32, ctypes.c_int64, ctypes.c_uint64,
                                ctypes.c_double, ctypes.c_float, ctypes.c_char_p)

SIGS = {
    # name: (restype, argtypes)
    "dtfrt_last_error": (S, []),
    "dtfrt_crc32c": (U32, [P, ctypes.c_size_t, U32]),
    "dtfrt_crc_mask": (U32, [U32]),
    # tensor bundle
    "dtfrt_bundle_writer_open": (P, [S, I]),
    "dtfrt_bundle_add": (I, [P, S, I, I, P, P, I64, I]),
    "dtfrt_bundle_add_strings": (I, [P, S, I, P, I, P, P, I]),
    "dtfrt_bundle_finish": (I, [P]),
    "dtfrt_bundle_reader_open": (P, [S]),
    "dtfrt_bundle_num_tensors": (I, [P]),
    "dtfrt_bundle_name": (S, [P, I]),
    "dtfrt_bundle_info": (I, [P, S, P, P, P, P]),
    "dtfrt_bundle_read": (I, [P, S, P, I64]),
    "dtfrt_bundle_reader_close": (None, [P]),
    # tfrecord / events
    "dtfrt_tfrecord_writer_open": (P, [S, I]),
    "dtfrt_tfrecord_write": (I, [P, P, U64]),
    "dtfrt_tfrecord_flush": (I, [P]),
    "dtfrt_tfrecord_writer_close": (None, [P]),
    "dtfrt_events_open": (P, [S]),
    "dtfrt_events_scalar": (I, [P, S, F, I64, D]),
    "dtfrt_events_summary": (I, [P, P, U64, I64, D]),
    "dtfrt_events_graph": (I, [P, P, U64, D]),
    "dtfrt_tfrecord_reader_open": (P, [S]),
    "dtfrt_tfrecord_next": (I, [P, P, P]),
    "dtfrt_tfrecord_reader_close": (None, [P]),
    # kv store
    "dtfrt_kv_server_start": (P, [S, I, P]),
    "dtfrt_kv_server_stop": (None, [P]),
    "dtfrt_kv_connect": (P, [S, I, I]),
    "dtfrt_kv_close": (None, [P]),
    "dtfrt_kv_set": (I, [P, S, P, U64]),
    "dtfrt_kv_get": (I, [P, S, I64, P]),
    "dtfrt_kv_result": (P, [P]),
    "dtfrt_kv_add": (I64, [P, S, I64]),
    "dtfrt_kv_check": (I, [P, S]),
    "dtfrt_kv_del": (I, [P, S]),
    "dtfrt_kv_wait_ge": (I, [P, S, I64, I64, P]),
    "dtfrt_kv_keys": (I, [P, S, P]),
    # parameter-server transport
    "dtfrt_ps_server_start": (P, [S, I, P]),
    "dtfrt_ps_register": (I, [P, I, P, U64]),
    "dtfrt_ps_lock": (I, [P, I]),
    "dtfrt_ps_unlock": (I, [P, I, I]),
    "dtfrt_ps_next_push": (I, [P, I, P, P, P, P]),
    "dtfrt_ps_push_done": (I, [P, I, I]),
    "dtfrt_ps_stats": (None, [P, P, P]),
    "dtfrt_ps_server_stop": (None, [P]),
    "dtfrt_ps_connect": (P, [S, I, I]),
    "dtfrt_ps_pull": (I, [P, I, U64, P, U64, P]),
    "dtfrt_ps_push": (I, [P, I, U64, P, U64, P]),
    "dtfrt_ps_var_bytes": (I64, [P, I]),
    "dtfrt_ps_close": (None, [P]),
    # intra-node PS mailbox + shared-memory regions (ps_mailbox.cc)
    "dtfrt_mbox_create": (P, [S, I]),
    "dtfrt_mbox_open": (P, [S, I]),
    "dtfrt_mbox_post": (I64, [P, I, I, U64]),
    "dtfrt_mbox_wait": (I, [P, I, I64, I]),
    "dtfrt_mbox_next": (I, [P, I, P, P, P, P]),
    "dtfrt_mbox_complete": (I, [P, I, I64, I]),
    "dtfrt_mbox_close": (None, [P, I]),
    "dtfrt_shmem_create": (P, [S, U64]),
    "dtfrt_shmem_open": (P, [S, U64, I]),
    "dtfrt_shmem_close": (None, [P, U64, S, I]),
    # shared-memory CPU all-reduce
    "dtfrt_shm_open": (P, [S, I, I, U64]),
    "dtfrt_shm_allreduce_f32": (I, [P, P, U64]),
    "dtfrt_shm_barrier": (I, [P]),
    "dtfrt_shm_close": (None, [P, I]),
    # RCCL communicator (rccl_comm.cc)
    "dtfrt_rccl_available": (I, [P]),
    "dtfrt_rccl_version": (I, []),
    "dtfrt_rccl_error_string": (S, [I]),
    "dtfrt_rccl_unique_id": (I, [P]),
    "dtfrt_rccl_comm_init": (P, [P, I, I, I, I, S, P]),
    "dtfrt_rccl_comm_destroy": (I, [P, I]),
    "dtfrt_rccl_comm_info": (I, [P, P, P, P, P]),
    "dtfrt_rccl_async_error": (I, [P]),
    "dtfrt_rccl_all_reduce": (I, [P, P, P, I64, I, I, P]),
    "dtfrt_rccl_reduce_scatter": (I, [P, P, P, I64, I, I, P]),
    "dtfrt_rccl_all_gather": (I, [P, P, P, I64, I, P]),
    "dtfrt_rccl_broadcast": (I, [P, P, P, I64, I, I, P]),
    "dtfrt_rccl_send": (I, [P, P, I64, I, I, P]),
    "dtfrt_rccl_recv": (I, [P, P, I64, I, I, P]),
    "dtfrt_rccl_group_start": (I, []),
    "dtfrt_rccl_group_end": (I, []),
}


def declare(lib):
    for name, (res, args) in SIGS.items():
        fn = getattr(lib, name, None)
        if fn is None:
            continue
        fn.restype = res
        fn.argtypes = args


def err(lib):
    e = lib.dtfrt_last_error()
    return e.decode() if e else "unknown error"
