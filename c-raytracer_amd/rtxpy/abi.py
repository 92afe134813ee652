"""ctypes mirror of include/rtx.h, include/rtx_scene.h and include/rtx_kat.h.

Test / bench plumbing only: the product boundary is the C-ABI in include/.
"""
import ctypes as C

RTX_OK = 0
RTX_ERR_ARG, RTX_ERR_HIP, RTX_ERR_NOMEM, RTX_ERR_SCENE, RTX_ERR_NODEV, RTX_ERR_STATE, RTX_ERR_IO = (
    -1, -2, -3, -4, -5, -6, -7)

RTX_SPHERE, RTX_TRIANGLE, RTX_PLANE = 0, 1, 2
RTX_TEX_UNIFORM, RTX_TEX_CHECKERBOARD, RTX_TEX_BRICK, RTX_TEX_NOISY_PERIODIC = 0, 1, 2, 3
RTX_PHONG, RTX_BLINN = 0, 1
RTX_GI_AMBIENT, RTX_GI_PATH = 0, 1
RTX_ATT_NONE, RTX_ATT_LIN, RTX_ATT_SQR = 0, 1, 2
RTX_RNG_COUNTER, RTX_RNG_CONST, RTX_RNG_STRAT = 0, 1, 2
RTX_U32_SAT, RTX_U32_WRAP = 0, 1

F3 = C.c_float * 3


class Material(C.Structure):
    _fields_ = [("id", C.c_int32), ("ks", F3), ("ka", F3), ("kr", F3), ("kt", F3), ("ke", F3),
                ("shininess", C.c_float), ("refractive_index", C.c_float), ("texture", C.c_int32),
                ("periodic", C.c_int32), ("color", F3 * 2), ("scale", C.c_float), ("mortar_width", C.c_float),
                ("noise_feature_scale", C.c_float), ("noise_scale", C.c_float), ("frequency_scale", C.c_float),
                ("emittant", C.c_int32), ("reflective", C.c_int32), ("transparent", C.c_int32)]


class Object(C.Structure):
    _fields_ = [("type", C.c_int32), ("material", C.c_int32), ("num_lights", C.c_uint32), ("epsilon", C.c_float),
                ("p0", F3), ("p1", F3), ("p2", F3), ("e1", F3), ("e2", F3), ("n", F3), ("radius", C.c_float),
                ("d", C.c_float)]


class Camera(C.Structure):
    _fields_ = [("position", F3), ("vectors", F3 * 3), ("fov", C.c_float), ("focal_length", C.c_float)]


class SceneDesc(C.Structure):
    _fields_ = [("num_materials", C.c_uint32), ("materials", C.POINTER(Material)), ("num_objects", C.c_uint32),
                ("objects", C.POINTER(Object)), ("num_emitters", C.c_uint32), ("emitters", C.POINTER(C.c_uint32)),
                ("ambient", F3), ("camera", Camera)]


class Frame(C.Structure):
    _fields_ = [("width", C.c_uint32), ("height", C.c_uint32), ("corner", F3), ("step_x", F3), ("step_y", F3),
                ("origin", F3)]


class Params(C.Structure):
    _fields_ = [("max_bounces", C.c_uint32), ("min_intensity_sqr", C.c_float), ("reflection", C.c_int32),
                ("gi", C.c_int32), ("samples", C.c_uint32), ("attenuation", C.c_int32),
                ("attenuation_offset", C.c_float), ("rng", C.c_int32), ("seed", C.c_uint64),
                ("u32conv", C.c_int32), ("tile_offset", C.c_uint32), ("tile_stride", C.c_uint32),
                ("count_traversal", C.c_int32)]


class Stats(C.Structure):
    _fields_ = [("closest_rays", C.c_uint64), ("shadow_rays", C.c_uint64), ("node_visits", C.c_uint64),
                ("tri_tests", C.c_uint64), ("sphere_tests", C.c_uint64), ("plane_tests", C.c_uint64),
                ("shadow_node_visits", C.c_uint64), ("shadow_tri_tests", C.c_uint64),
                ("shadow_sphere_tests", C.c_uint64), ("shadow_plane_tests", C.c_uint64),
                ("shade_points", C.c_uint64), ("kernel_ms", C.c_double), ("trace_ms", C.c_double),
                ("shadow_ms", C.c_double), ("accum_ms", C.c_double), ("sort_ms", C.c_double), ("build_ms", C.c_double),
                ("bvh_nodes", C.c_uint32),
                ("bvh_depth", C.c_uint32), ("bvh_prims", C.c_uint32), ("waves", C.c_uint32),
                ("chunks", C.c_uint32), ("builder", C.c_uint32),
                ("shadow_box_tests", C.c_uint64), ("shadow_global_box_tests", C.c_uint64),
                ("shadow_wave_steps", C.c_uint64), ("shadow_wave_walks", C.c_uint64),
                ("wide_nodes", C.c_uint32), ("wide_depth", C.c_uint32), ("shadow_leaf_rounds", C.c_uint64),
                ("gather_ms", C.c_double), ("devices", C.c_uint32), ("pad_", C.c_uint32),
                ("shadow_uniform_steps", C.c_uint64), ("shadow_walk", C.c_uint32), ("wide_entries", C.c_uint32),
                ("trace_walk", C.c_uint32), ("pad2_", C.c_uint32), ("tree_rotated", C.c_uint32),
                ("pad3_", C.c_uint32), ("frame_cost", C.c_double), ("frame_ms", C.c_double),
                ("upload_copy_ms", C.c_double), ("transport", C.c_uint32), ("peer_access", C.c_uint32),
                ("far_closest_rays", C.c_uint64), ("far_shadow_rays", C.c_uint64),
                ("shadow_stack_spills", C.c_uint64), ("shadow_cone_clear", C.c_uint64)]


RTX_TRANSPORT_NONE, RTX_TRANSPORT_RCCL, RTX_TRANSPORT_LOOPBACK, RTX_TRANSPORT_RCCL_SELF = 0, 1, 2, 3


class GroupMember(C.Structure):
    _fields_ = [("device", C.c_int32), ("comm_count", C.c_int32), ("comm_rank", C.c_int32), ("comm_device", C.c_int32),
                ("can_access_peer0", C.c_uint32), ("peer0_can_access", C.c_uint32), ("peer_enabled", C.c_uint32),
                ("transport", C.c_uint32), ("pci_bus_id", C.c_char * 32)]


RTX_BUILD_SAH_HOST, RTX_BUILD_LBVH_GPU, RTX_BUILD_PLOC_GPU, RTX_BUILD_SAH_GPU = 0, 1, 2, 3
RTX_WALK_AUTO, RTX_WALK_BVH2, RTX_WALK_W8, RTX_WALK_LINEAR = -1, 0, 2, 3
WALK_NAMES = {RTX_WALK_BVH2: "bvh2", RTX_WALK_W8: "w8", RTX_WALK_LINEAR: "linear"}
RTX_SHADOW_LINEAR_MAX = 8
RTX_FRAME_AUTO, RTX_FRAME_WORLD = 0, 1
RTX_OPT_SHADOW_WALK, RTX_OPT_BVH_LEAF, RTX_OPT_SPSORT, RTX_OPT_SHADOW_SLOT, RTX_OPT_SHADOW_GRAB, \
    RTX_OPT_SHADOW_LDS_STACK, RTX_OPT_TRACE_WALK, RTX_OPT_TREE_FRAME, RTX_OPT_CHUNK_TILES, \
    RTX_OPT_SP_PER_TILE, RTX_OPT_SHADOW_CULL = 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11
RTX_DOF_NONE, RTX_DOF_SCALE_BIAS, RTX_DOF_CAMERA = 0, 1, 2
RTX_FALLOFF_QUAD, RTX_FALLOFF_LIN, RTX_FALLOFF_INV_QUAD = 0, 1, 2


class Post(C.Structure):
    _fields_ = [("brighten", C.c_int32), ("brighten_factor", C.c_float), ("dof", C.c_int32),
                ("dof_scale", C.c_float), ("dof_bias", C.c_float), ("aperture", C.c_float),
                ("focal_length", C.c_float), ("plane_in_focus", C.c_float), ("mist", C.c_int32),
                ("mist_start", C.c_float), ("mist_depth", C.c_float), ("mist_falloff", C.c_int32),
                ("mist_color", F3)]


# include/rtx_kat.h
KAT_MOLLER, KAT_SPHERE, KAT_PLANE, KAT_SLAB, KAT_NOISE, KAT_TEXTURE, KAT_SPH_LIGHT, KAT_TRI_LIGHT, \
    KAT_MORTON, KAT_U32, KAT_GI_DIR, KAT_REFRACT, KAT_ANY_TRI, KAT_SPH_LIGHT_SH, KAT_BOX_Q, KAT_SPEC_POW, \
    KAT_BOX_Q8 = range(17)
KAT_IN = [16, 11, 11, 13, 3, 16, 9, 11, 3, 1, 6, 7, 17, 9, 19, 2, 25]
KAT_OUT = [2, 5, 5, 3, 1, 3, 3, 3, 1, 2, 3, 3, 1, 3, 2, 1, 2]
KAT_NAMES = ["moller", "sphere", "plane", "slab", "noise", "texture", "sph_light", "tri_light", "morton", "u32",
             "gi_dir", "refract", "any_tri", "sph_light_sh", "box_q", "spec_pow", "box_q8"]

# symbols include/rtx.h declares (checked by tests/test_abi.py)
RTX_SYMBOLS = ["rtx_params_default", "rtx_device_count", "rtx_open", "rtx_upload_scene", "rtx_render",
               "rtx_render_device", "rtx_get_stats", "rtx_close", "rtx_last_error", "rtx_kat", "rtx_postprocess",
               "rtx_postprocess_device", "rtx_set_builder", "rtx_set_option", "rtx_group_open", "rtx_group_open_loopback", "rtx_group_open_rccl_self", "rtx_group_size", "rtx_read_wide_tree",
               "rtx_group_set_builder", "rtx_group_set_option", "rtx_group_upload_scene", "rtx_group_render", "rtx_group_get_stats", "rtx_group_device_stats",
               "rtx_group_member_info", "rtx_group_close", "rtx_tile_pack_count", "rtx_tile_pack_host", "rtx_tile_unpack_host",
               "rtx_tile_pack_device", "rtx_tile_unpack_device", "rtx_tree_frame"]
RTX_SCENE_SYMBOLS = ["rtx_scene_load", "rtx_scene_parse", "rtx_scene_desc_of", "rtx_scene_num_json_objects",
                     "rtx_scene_free", "rtx_scene_last_error", "rtx_frame_setup", "rtx_tiff_write", "rtx_hash_djb",
                     "rtx_params_from_argv", "rtx_stl_write", "rtx_tiff_read_raw", "rtx_buffer_free",
                     "rtx_post_from_argv"]


def declare_scene(lib):
    lib.rtx_scene_load.argtypes = [C.c_char_p, C.c_char_p, C.c_char_p, C.POINTER(C.c_void_p)]
    lib.rtx_scene_load.restype = C.c_int
    lib.rtx_scene_parse.argtypes = [C.c_char_p, C.c_size_t, C.c_char_p, C.c_char_p, C.c_char_p,
                                    C.POINTER(C.c_void_p)]
    lib.rtx_scene_parse.restype = C.c_int
    lib.rtx_scene_desc_of.argtypes = [C.c_void_p]
    lib.rtx_scene_desc_of.restype = C.POINTER(SceneDesc)
    lib.rtx_scene_num_json_objects.argtypes = [C.c_void_p]
    lib.rtx_scene_num_json_objects.restype = C.c_uint32
    lib.rtx_scene_free.argtypes = [C.c_void_p]
    lib.rtx_scene_free.restype = None
    lib.rtx_scene_last_error.argtypes = []
    lib.rtx_scene_last_error.restype = C.c_char_p
    lib.rtx_frame_setup.argtypes = [C.POINTER(Camera), C.c_uint32, C.c_uint32, C.POINTER(Frame)]
    lib.rtx_frame_setup.restype = C.c_int
    lib.rtx_tiff_write.argtypes = [C.c_char_p, C.c_uint32, C.c_uint32, C.c_void_p, C.c_void_p, C.c_int]
    lib.rtx_tiff_write.restype = C.c_int
    lib.rtx_hash_djb.argtypes = [C.c_char_p]
    lib.rtx_hash_djb.restype = C.c_uint32
    lib.rtx_params_from_argv.argtypes = [C.c_int, C.POINTER(C.c_char_p), C.POINTER(Params)]
    lib.rtx_params_from_argv.restype = None
    lib.rtx_stl_write.argtypes = [C.c_char_p, C.c_uint32, C.c_void_p]
    lib.rtx_stl_write.restype = C.c_int
    lib.rtx_tiff_read_raw.argtypes = [C.c_char_p, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32),
                                      C.POINTER(C.c_void_p), C.POINTER(C.c_void_p)]
    lib.rtx_tiff_read_raw.restype = C.c_int
    lib.rtx_buffer_free.argtypes = [C.c_void_p]
    lib.rtx_buffer_free.restype = None
    lib.rtx_post_from_argv.argtypes = [C.c_int, C.POINTER(C.c_char_p), C.POINTER(Post)]
    lib.rtx_post_from_argv.restype = C.c_int


def declare_rtx(lib):
    lib.rtx_params_default.argtypes = [C.POINTER(Params)]
    lib.rtx_params_default.restype = None
    lib.rtx_device_count.argtypes = [C.POINTER(C.c_int)]
    lib.rtx_device_count.restype = C.c_int
    lib.rtx_open.argtypes = [C.c_int, C.POINTER(C.c_void_p)]
    lib.rtx_open.restype = C.c_int
    lib.rtx_upload_scene.argtypes = [C.c_void_p, C.POINTER(SceneDesc)]
    lib.rtx_upload_scene.restype = C.c_int
    lib.rtx_render.argtypes = [C.c_void_p, C.POINTER(Frame), C.POINTER(Params), C.c_void_p, C.c_void_p]
    lib.rtx_render.restype = C.c_int
    lib.rtx_render_device.argtypes = [C.c_void_p, C.POINTER(Frame), C.POINTER(Params), C.c_void_p, C.c_void_p,
                                      C.c_void_p]
    lib.rtx_render_device.restype = C.c_int
    lib.rtx_get_stats.argtypes = [C.c_void_p, C.POINTER(Stats)]
    lib.rtx_get_stats.restype = C.c_int
    lib.rtx_close.argtypes = [C.c_void_p]
    lib.rtx_close.restype = None
    lib.rtx_last_error.argtypes = []
    lib.rtx_last_error.restype = C.c_char_p
    lib.rtx_kat.argtypes = [C.c_int, C.c_uint32, C.c_void_p, C.c_void_p, C.POINTER(Params)]
    lib.rtx_kat.restype = C.c_int
    lib.rtx_set_builder.argtypes = [C.c_void_p, C.c_int]
    lib.rtx_set_builder.restype = C.c_int
    lib.rtx_set_option.argtypes = [C.c_void_p, C.c_int, C.c_int64]
    lib.rtx_set_option.restype = C.c_int
    lib.rtx_group_set_option.argtypes = [C.c_void_p, C.c_int, C.c_int64]
    lib.rtx_group_set_option.restype = C.c_int
    lib.rtx_postprocess.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.POINTER(Post), C.c_void_p, C.c_void_p]
    lib.rtx_postprocess.restype = C.c_int
    lib.rtx_postprocess_device.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.POINTER(Post), C.c_void_p,
                                           C.c_void_p, C.c_void_p]
    lib.rtx_postprocess_device.restype = C.c_int
    lib.rtx_group_open.argtypes = [C.c_int, C.c_void_p, C.POINTER(C.c_void_p)]
    lib.rtx_group_open.restype = C.c_int
    lib.rtx_read_wide_tree.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.POINTER(C.c_uint32), C.c_void_p]
    lib.rtx_read_wide_tree.restype = C.c_int
    lib.rtx_group_open_loopback.argtypes = [C.c_int, C.c_int, C.POINTER(C.c_void_p)]
    lib.rtx_group_open_loopback.restype = C.c_int
    lib.rtx_group_open_rccl_self.argtypes = [C.c_int, C.POINTER(C.c_void_p)]
    lib.rtx_group_open_rccl_self.restype = C.c_int
    lib.rtx_group_size.argtypes = [C.c_void_p]
    lib.rtx_group_size.restype = C.c_int
    lib.rtx_group_set_builder.argtypes = [C.c_void_p, C.c_int]
    lib.rtx_group_set_builder.restype = C.c_int
    lib.rtx_group_upload_scene.argtypes = [C.c_void_p, C.POINTER(SceneDesc)]
    lib.rtx_group_upload_scene.restype = C.c_int
    lib.rtx_group_render.argtypes = [C.c_void_p, C.POINTER(Frame), C.POINTER(Params), C.c_void_p, C.c_void_p]
    lib.rtx_group_render.restype = C.c_int
    lib.rtx_group_get_stats.argtypes = [C.c_void_p, C.POINTER(Stats)]
    lib.rtx_group_get_stats.restype = C.c_int
    lib.rtx_group_device_stats.argtypes = [C.c_void_p, C.c_int, C.POINTER(Stats)]
    lib.rtx_group_device_stats.restype = C.c_int
    lib.rtx_group_member_info.argtypes = [C.c_void_p, C.c_int, C.POINTER(GroupMember)]
    lib.rtx_group_member_info.restype = C.c_int
    lib.rtx_group_close.argtypes = [C.c_void_p]
    lib.rtx_group_close.restype = None
    lib.rtx_tile_pack_count.argtypes = [C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32]
    lib.rtx_tile_pack_count.restype = C.c_size_t
    lib.rtx_tile_pack_host.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                       C.c_void_p]
    lib.rtx_tile_pack_host.restype = C.c_int
    lib.rtx_tile_unpack_host.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_void_p,
                                         C.c_void_p]
    lib.rtx_tile_unpack_host.restype = C.c_int
    lib.rtx_tile_pack_device.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32,
                                         C.c_uint32, C.c_void_p, C.c_void_p]
    lib.rtx_tile_pack_device.restype = C.c_int
    lib.rtx_tile_unpack_device.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                           C.c_void_p, C.c_void_p, C.c_void_p]
    lib.rtx_tile_unpack_device.restype = C.c_int
    lib.rtx_tree_frame.argtypes = [C.POINTER(SceneDesc), C.POINTER(C.c_int), C.c_void_p, C.c_void_p,
                                   C.POINTER(C.c_double)]
    lib.rtx_tree_frame.restype = C.c_int


def declare_oracle(lib):
    lib.rtx_oracle_params_default.argtypes = [C.POINTER(Params)]
    lib.rtx_oracle_params_default.restype = None
    lib.rtx_oracle_render.argtypes = [C.POINTER(SceneDesc), C.POINTER(Frame), C.POINTER(Params), C.c_void_p,
                                      C.c_void_p, C.POINTER(C.c_uint64), C.c_int]
    lib.rtx_oracle_render.restype = C.c_int
    lib.rtx_oracle_kat.argtypes = [C.c_int, C.c_uint32, C.c_void_p, C.c_void_p, C.POINTER(Params)]
    lib.rtx_oracle_kat.restype = C.c_int
    lib.rtx_oracle_primary.argtypes = [C.POINTER(SceneDesc), C.POINTER(Frame), C.c_void_p, C.c_void_p, C.c_int]
    lib.rtx_oracle_primary.restype = C.c_int
