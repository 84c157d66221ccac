/*
 * ggml_abi.h — binary-layout mirror of the ggml 0.9.5 structures that cross the
 * backend boundary, written from the reference headers' documented layout so the
 * MI355X backend builds with no dependency on the reference tree.
 *
 *   struct ggml_tensor        ggml/include/ggml.h:655-687   (sizeof 336)
 *   struct ggml_cgraph        ggml/src/ggml-impl.h:323-337  (sizeof 88)
 *   backend vtables           ggml/src/ggml-backend-impl.h:17-210
 *   dev props / caps          ggml/include/ggml-backend.h:150-171
 *   enum ggml_type            ggml/include/ggml.h:389-431
 *   enum ggml_op              ggml/include/ggml.h:469-576
 *   enum ggml_unary_op/glu_op ggml/include/ggml.h:578-614
 *
 * Only the members the backend touches are given meaningful names; every offset
 * is pinned by static_assert below and re-checked against the real headers by
 * tests/test_abi_cpu.py (test_abi_layout_matches_reference: ggml_tensor and enums;
 * test_vtable_layout_matches_reference: every backend vtable and the structs embedding
 * them, ggml-backend-impl.h:17-210 — probes compiled against /root/reference when present).
 */
#pragma once

#include <stddef.h>
#include <stdint.h>
#include <stdbool.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GGML_MAX_DIMS        4
#define GGML_MAX_SRC         10
#define GGML_MAX_OP_PARAMS   64
#define GGML_MAX_NAME        64
#define GGML_BACKEND_API_VERSION 2

#define GGML_ROPE_TYPE_NORMAL 0
#define GGML_ROPE_TYPE_NEOX   2
#define GGML_ROPE_TYPE_MROPE  8
#define GGML_ROPE_TYPE_VISION 24

#define QK_K   256
#define QK4_0  32
#define QK8_0  32
#define QK8_1  32

enum ggml_status {
    GGML_STATUS_ALLOC_FAILED = -2,
    GGML_STATUS_FAILED       = -1,
    GGML_STATUS_SUCCESS      = 0,
    GGML_STATUS_ABORTED      = 1,
};

enum ggml_type {
    GGML_TYPE_F32  = 0,  GGML_TYPE_F16  = 1,  GGML_TYPE_Q4_0 = 2,  GGML_TYPE_Q4_1 = 3,
    GGML_TYPE_Q5_0 = 6,  GGML_TYPE_Q5_1 = 7,  GGML_TYPE_Q8_0 = 8,  GGML_TYPE_Q8_1 = 9,
    GGML_TYPE_Q2_K = 10, GGML_TYPE_Q3_K = 11, GGML_TYPE_Q4_K = 12, GGML_TYPE_Q5_K = 13,
    GGML_TYPE_Q6_K = 14, GGML_TYPE_Q8_K = 15,
    GGML_TYPE_I8   = 24, GGML_TYPE_I16  = 25, GGML_TYPE_I32  = 26, GGML_TYPE_I64  = 27,
    GGML_TYPE_F64  = 28, GGML_TYPE_BF16 = 30,
    GGML_TYPE_COUNT = 40,
};

enum ggml_prec { GGML_PREC_DEFAULT = 0, GGML_PREC_F32 = 10 };

/* Order matters: values are positional (ggml.h:469-576). */
enum ggml_op {
    GGML_OP_NONE = 0,
    GGML_OP_DUP, GGML_OP_ADD, GGML_OP_ADD_ID, GGML_OP_ADD1, GGML_OP_ACC, GGML_OP_SUB,
    GGML_OP_MUL, GGML_OP_DIV, GGML_OP_SQR, GGML_OP_SQRT, GGML_OP_LOG, GGML_OP_SIN,
    GGML_OP_COS, GGML_OP_SUM, GGML_OP_SUM_ROWS, GGML_OP_CUMSUM, GGML_OP_MEAN,
    GGML_OP_ARGMAX, GGML_OP_COUNT_EQUAL, GGML_OP_REPEAT, GGML_OP_REPEAT_BACK,
    GGML_OP_CONCAT, GGML_OP_SILU_BACK, GGML_OP_NORM, GGML_OP_RMS_NORM,
    GGML_OP_RMS_NORM_BACK, GGML_OP_GROUP_NORM, GGML_OP_L2_NORM,
    GGML_OP_MUL_MAT, GGML_OP_MUL_MAT_ID, GGML_OP_OUT_PROD,
    GGML_OP_SCALE, GGML_OP_SET, GGML_OP_CPY, GGML_OP_CONT, GGML_OP_RESHAPE,
    GGML_OP_VIEW, GGML_OP_PERMUTE, GGML_OP_TRANSPOSE, GGML_OP_GET_ROWS,
    GGML_OP_GET_ROWS_BACK, GGML_OP_SET_ROWS, GGML_OP_DIAG, GGML_OP_DIAG_MASK_INF,
    GGML_OP_DIAG_MASK_ZERO, GGML_OP_SOFT_MAX, GGML_OP_SOFT_MAX_BACK, GGML_OP_ROPE,
    GGML_OP_ROPE_BACK, GGML_OP_CLAMP, GGML_OP_CONV_TRANSPOSE_1D, GGML_OP_IM2COL,
    GGML_OP_IM2COL_BACK, GGML_OP_IM2COL_3D, GGML_OP_CONV_2D, GGML_OP_CONV_3D,
    GGML_OP_CONV_2D_DW, GGML_OP_CONV_TRANSPOSE_2D, GGML_OP_POOL_1D, GGML_OP_POOL_2D,
    GGML_OP_POOL_2D_BACK, GGML_OP_UPSCALE, GGML_OP_PAD, GGML_OP_PAD_REFLECT_1D,
    GGML_OP_ROLL, GGML_OP_ARANGE, GGML_OP_TIMESTEP_EMBEDDING, GGML_OP_ARGSORT,
    GGML_OP_TOP_K, GGML_OP_LEAKY_RELU, GGML_OP_TRI, GGML_OP_FILL,
    GGML_OP_FLASH_ATTN_EXT, GGML_OP_FLASH_ATTN_BACK, GGML_OP_SSM_CONV,
    GGML_OP_SSM_SCAN, GGML_OP_WIN_PART, GGML_OP_WIN_UNPART, GGML_OP_GET_REL_POS,
    GGML_OP_ADD_REL_POS, GGML_OP_RWKV_WKV6, GGML_OP_GATED_LINEAR_ATTN,
    GGML_OP_RWKV_WKV7, GGML_OP_SOLVE_TRI,
    GGML_OP_UNARY,
    GGML_OP_MAP_CUSTOM1, GGML_OP_MAP_CUSTOM2, GGML_OP_MAP_CUSTOM3, GGML_OP_CUSTOM,
    GGML_OP_CROSS_ENTROPY_LOSS, GGML_OP_CROSS_ENTROPY_LOSS_BACK,
    GGML_OP_OPT_STEP_ADAMW, GGML_OP_OPT_STEP_SGD,
    GGML_OP_GLU,
    GGML_OP_COUNT,
};

enum ggml_unary_op {
    GGML_UNARY_OP_ABS, GGML_UNARY_OP_SGN, GGML_UNARY_OP_NEG, GGML_UNARY_OP_STEP,
    GGML_UNARY_OP_TANH, GGML_UNARY_OP_ELU, GGML_UNARY_OP_RELU, GGML_UNARY_OP_SIGMOID,
    GGML_UNARY_OP_GELU, GGML_UNARY_OP_GELU_QUICK, GGML_UNARY_OP_SILU,
    GGML_UNARY_OP_HARDSWISH, GGML_UNARY_OP_HARDSIGMOID, GGML_UNARY_OP_EXP,
    GGML_UNARY_OP_EXPM1, GGML_UNARY_OP_SOFTPLUS, GGML_UNARY_OP_GELU_ERF,
    GGML_UNARY_OP_XIELU, GGML_UNARY_OP_FLOOR, GGML_UNARY_OP_CEIL,
    GGML_UNARY_OP_ROUND, GGML_UNARY_OP_TRUNC,
    GGML_UNARY_OP_COUNT,
};

enum ggml_glu_op {
    GGML_GLU_OP_REGLU, GGML_GLU_OP_GEGLU, GGML_GLU_OP_SWIGLU, GGML_GLU_OP_SWIGLU_OAI,
    GGML_GLU_OP_GEGLU_ERF, GGML_GLU_OP_GEGLU_QUICK,
    GGML_GLU_OP_COUNT,
};

enum ggml_sort_order { GGML_SORT_ORDER_ASC = 0, GGML_SORT_ORDER_DESC = 1 };

enum ggml_tensor_flag {
    GGML_TENSOR_FLAG_INPUT   = 1,
    GGML_TENSOR_FLAG_OUTPUT  = 2,
    GGML_TENSOR_FLAG_PARAM   = 4,
    GGML_TENSOR_FLAG_LOSS    = 8,
    GGML_TENSOR_FLAG_COMPUTE = 16,
};

struct ggml_backend_buffer;

struct ggml_tensor {
    enum ggml_type type;
    struct ggml_backend_buffer * buffer;
    int64_t ne[GGML_MAX_DIMS];
    size_t  nb[GGML_MAX_DIMS];
    enum ggml_op op;
    int32_t op_params[GGML_MAX_OP_PARAMS / sizeof(int32_t)];
    int32_t flags;
    struct ggml_tensor * src[GGML_MAX_SRC];
    struct ggml_tensor * view_src;
    size_t view_offs;
    void * data;
    char name[GGML_MAX_NAME];
    void * extra;
    char padding[8];
};

typedef uint32_t ggml_bitset_t;

struct ggml_hash_set {
    size_t size;
    ggml_bitset_t * used;
    struct ggml_tensor ** keys;
};

enum ggml_cgraph_eval_order { GGML_CGRAPH_EVAL_ORDER_LEFT_TO_RIGHT = 0 };

struct ggml_cgraph {
    int size;
    int n_nodes;
    int n_leafs;
    struct ggml_tensor ** nodes;
    struct ggml_tensor ** grads;
    struct ggml_tensor ** grad_accs;
    struct ggml_tensor ** leafs;
    int32_t * use_counts;
    struct ggml_hash_set visited_hash_set;
    enum ggml_cgraph_eval_order order;
};

typedef uint8_t ggml_guid[16];
typedef ggml_guid * ggml_guid_t;

typedef struct ggml_backend_buffer_type * ggml_backend_buffer_type_t;
typedef struct ggml_backend_buffer      * ggml_backend_buffer_t;
typedef struct ggml_backend_event       * ggml_backend_event_t;
typedef struct ggml_backend             * ggml_backend_t;
typedef void                            * ggml_backend_graph_plan_t;
typedef struct ggml_backend_reg         * ggml_backend_reg_t;
typedef struct ggml_backend_device      * ggml_backend_dev_t;

enum ggml_backend_buffer_usage {
    GGML_BACKEND_BUFFER_USAGE_ANY = 0,
    GGML_BACKEND_BUFFER_USAGE_WEIGHTS = 1,
    GGML_BACKEND_BUFFER_USAGE_COMPUTE = 2,
};

enum ggml_backend_dev_type {
    GGML_BACKEND_DEVICE_TYPE_CPU,
    GGML_BACKEND_DEVICE_TYPE_GPU,
    GGML_BACKEND_DEVICE_TYPE_IGPU,
    GGML_BACKEND_DEVICE_TYPE_ACCEL,
};

struct ggml_backend_dev_caps {
    bool async;
    bool host_buffer;
    bool buffer_from_host_ptr;
    bool events;
};

struct ggml_backend_dev_props {
    const char * name;
    const char * description;
    size_t memory_free;
    size_t memory_total;
    enum ggml_backend_dev_type type;
    const char * device_id;
    struct ggml_backend_dev_caps caps;
};

struct ggml_backend_buffer_type_i {
    const char *          (*get_name)      (ggml_backend_buffer_type_t buft);
    ggml_backend_buffer_t (*alloc_buffer)  (ggml_backend_buffer_type_t buft, size_t size);
    size_t                (*get_alignment) (ggml_backend_buffer_type_t buft);
    size_t                (*get_max_size)  (ggml_backend_buffer_type_t buft);
    size_t                (*get_alloc_size)(ggml_backend_buffer_type_t buft, const struct ggml_tensor * tensor);
    bool                  (*is_host)       (ggml_backend_buffer_type_t buft);
};

struct ggml_backend_buffer_type {
    struct ggml_backend_buffer_type_i iface;
    ggml_backend_dev_t device;
    void * context;
};

struct ggml_backend_buffer_i {
    void             (*free_buffer)  (ggml_backend_buffer_t buffer);
    void *           (*get_base)     (ggml_backend_buffer_t buffer);
    enum ggml_status (*init_tensor)  (ggml_backend_buffer_t buffer, struct ggml_tensor * tensor);
    void             (*memset_tensor)(ggml_backend_buffer_t buffer, struct ggml_tensor * tensor, uint8_t value, size_t offset, size_t size);
    void             (*set_tensor)   (ggml_backend_buffer_t buffer, struct ggml_tensor * tensor, const void * data, size_t offset, size_t size);
    void             (*get_tensor)   (ggml_backend_buffer_t buffer, const struct ggml_tensor * tensor, void * data, size_t offset, size_t size);
    bool             (*cpy_tensor)   (ggml_backend_buffer_t buffer, const struct ggml_tensor * src, struct ggml_tensor * dst);
    void             (*clear)        (ggml_backend_buffer_t buffer, uint8_t value);
    void             (*reset)        (ggml_backend_buffer_t buffer);
};

struct ggml_backend_buffer {
    struct ggml_backend_buffer_i iface;
    ggml_backend_buffer_type_t buft;
    void * context;
    size_t size;
    enum ggml_backend_buffer_usage usage;
};

struct ggml_backend_i {
    const char * (*get_name)(ggml_backend_t backend);
    void (*free)(ggml_backend_t backend);
    void (*set_tensor_async)(ggml_backend_t backend, struct ggml_tensor * tensor, const void * data, size_t offset, size_t size);
    void (*get_tensor_async)(ggml_backend_t backend, const struct ggml_tensor * tensor, void * data, size_t offset, size_t size);
    bool (*cpy_tensor_async)(ggml_backend_t backend_src, ggml_backend_t backend_dst, const struct ggml_tensor * src, struct ggml_tensor * dst);
    void (*synchronize)(ggml_backend_t backend);
    ggml_backend_graph_plan_t (*graph_plan_create) (ggml_backend_t backend, const struct ggml_cgraph * cgraph);
    void                      (*graph_plan_free)   (ggml_backend_t backend, ggml_backend_graph_plan_t plan);
    void                      (*graph_plan_update) (ggml_backend_t backend, ggml_backend_graph_plan_t plan, const struct ggml_cgraph * cgraph);
    enum ggml_status          (*graph_plan_compute)(ggml_backend_t backend, ggml_backend_graph_plan_t plan);
    enum ggml_status          (*graph_compute)     (ggml_backend_t backend, struct ggml_cgraph * cgraph);
    void (*event_record)(ggml_backend_t backend, ggml_backend_event_t event);
    void (*event_wait)  (ggml_backend_t backend, ggml_backend_event_t event);
    void (*graph_optimize)(ggml_backend_t backend, struct ggml_cgraph * cgraph);
};

struct ggml_backend {
    ggml_guid_t guid;
    struct ggml_backend_i iface;
    ggml_backend_dev_t device;
    void * context;
};

struct ggml_backend_event {
    struct ggml_backend_device * device;
    void * context;
};

struct ggml_backend_device_i {
    const char * (*get_name)(ggml_backend_dev_t dev);
    const char * (*get_description)(ggml_backend_dev_t dev);
    void         (*get_memory)(ggml_backend_dev_t dev, size_t * free, size_t * total);
    enum ggml_backend_dev_type (*get_type)(ggml_backend_dev_t dev);
    void (*get_props)(ggml_backend_dev_t dev, struct ggml_backend_dev_props * props);
    ggml_backend_t (*init_backend)(ggml_backend_dev_t dev, const char * params);
    ggml_backend_buffer_type_t (*get_buffer_type)(ggml_backend_dev_t dev);
    ggml_backend_buffer_type_t (*get_host_buffer_type)(ggml_backend_dev_t dev);
    ggml_backend_buffer_t (*buffer_from_host_ptr)(ggml_backend_dev_t dev, void * ptr, size_t size, size_t max_tensor_size);
    bool (*supports_op)(ggml_backend_dev_t dev, const struct ggml_tensor * op);
    bool (*supports_buft)(ggml_backend_dev_t dev, ggml_backend_buffer_type_t buft);
    bool (*offload_op)(ggml_backend_dev_t dev, const struct ggml_tensor * op);
    ggml_backend_event_t (*event_new)        (ggml_backend_dev_t dev);
    void                 (*event_free)       (ggml_backend_dev_t dev, ggml_backend_event_t event);
    void                 (*event_synchronize)(ggml_backend_dev_t dev, ggml_backend_event_t event);
};

struct ggml_backend_device {
    struct ggml_backend_device_i iface;
    ggml_backend_reg_t reg;
    void * context;
};

struct ggml_backend_reg_i {
    const char *       (*get_name)(ggml_backend_reg_t reg);
    size_t             (*get_device_count)(ggml_backend_reg_t reg);
    ggml_backend_dev_t (*get_device)(ggml_backend_reg_t reg, size_t index);
    void *             (*get_proc_address)(ggml_backend_reg_t reg, const char * name);
};

struct ggml_backend_reg {
    int api_version;
    struct ggml_backend_reg_i iface;
    void * context;
};

typedef bool (*ggml_abort_callback)(void * data);

struct ggml_backend_feature {
    const char * name;
    const char * value;
};

#ifdef __cplusplus
}  /* extern "C" */

static_assert(sizeof(struct ggml_tensor) == 336, "ggml_tensor layout");
static_assert(offsetof(struct ggml_tensor, ne) == 16, "ggml_tensor.ne");
static_assert(offsetof(struct ggml_tensor, nb) == 48, "ggml_tensor.nb");
static_assert(offsetof(struct ggml_tensor, op) == 80, "ggml_tensor.op");
static_assert(offsetof(struct ggml_tensor, op_params) == 84, "ggml_tensor.op_params");
static_assert(offsetof(struct ggml_tensor, flags) == 148, "ggml_tensor.flags");
static_assert(offsetof(struct ggml_tensor, src) == 152, "ggml_tensor.src");
static_assert(offsetof(struct ggml_tensor, view_src) == 232, "ggml_tensor.view_src");
static_assert(offsetof(struct ggml_tensor, data) == 248, "ggml_tensor.data");
static_assert(offsetof(struct ggml_tensor, name) == 256, "ggml_tensor.name");
static_assert(offsetof(struct ggml_tensor, extra) == 320, "ggml_tensor.extra");
static_assert(sizeof(struct ggml_cgraph) == 88, "ggml_cgraph layout");
static_assert(offsetof(struct ggml_cgraph, nodes) == 16, "ggml_cgraph.nodes");
static_assert(GGML_OP_MUL_MAT == 29 && GGML_OP_GLU == 94 && GGML_OP_COUNT == 95, "ggml_op numbering");
static_assert(GGML_OP_FLASH_ATTN_EXT == 73 && GGML_OP_UNARY == 85, "ggml_op numbering");
#endif
