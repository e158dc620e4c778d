/*
 * capf_gpu.h — C-ABI of the MI355X relational backend for okapi-relational.
 *
 * This is the drop-in boundary that replaces the Flink implementation of the
 * okapi `Table[T]` SPI.  Every entry point below corresponds to one method of
 *
 *   trait Table[T <: Table[T]] extends CypherTable
 *     okapi-relational/src/main/scala/org/opencypher/okapi/relational/api/table/Table.scala:43-178
 *   trait CypherTable
 *     okapi-api/src/main/scala/org/opencypher/okapi/api/table/CypherTable.scala:41-70
 *
 * as implemented today by FlinkTable
 *     flink-cypher/src/main/scala/org/opencypher/flink/impl/table/FlinkTable.scala:49-199
 *
 * (citations are relative to the reference checkout).  A JVM shim
 * (`GpuTable extends Table[GpuTable]`) binds these
 * functions 1:1 over JNI; the Python host layer in
 * cypher-for-apache-flink_amd/table.py binds them over ctypes.
 *
 * Conventions
 *  - Tables are immutable, reference-counted handles.  Every operation returns
 *    a NEW handle (Table.scala: "every op returns a new T"); the caller owns it
 *    and must capf_table_release() it.  Column buffers are shared between
 *    handles, so select/drop/alias are metadata-only.
 *  - Evaluation is lazy, exactly like the Flink Table API: operations build a
 *    plan DAG; nothing runs on the GPU until capf_table_size / capf_table_download
 *    (FlinkTable.scala:57-61, CAPFRecords.scala:142-144).  This is what lets
 *    `group(∅, count(*))` over an Expand join chain run as a fused,
 *    factorised count instead of materialising ~1e12 joined rows.
 *  - Every function returns CAPF_OK (0) or a negative status.  The message
 *    is available from capf_last_error() (thread-local) and the kind from
 *    capf_last_error_kind(); the shim rethrows the matching
 *    okapi.impl.exception (okapi-api/.../impl/exception/InternalException.scala:36-65).
 *  - Column names are arbitrary caller strings (RecordHeader column names,
 *    okapi-relational/.../impl/table/RecordHeader.scala:299-318).
 *  - Logical types follow the Flink type mapping
 *    (flink-cypher/.../impl/convert/FlinkConversions.scala:43-117):
 *    CTInteger / node / relationship ids → INT64, CTFloat → FLOAT64,
 *    CTBoolean → BOOL, CTString → STRING (dictionary codes, see capf_string_*).
 */
#ifndef CAPF_GPU_H
#define CAPF_GPU_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CAPF_ABI_VERSION 1

typedef struct capf_session capf_session;
typedef struct capf_table capf_table;
typedef int32_t capf_status;

/* status codes */
enum {
  CAPF_OK = 0,
  CAPF_ERR_ILLEGAL_ARGUMENT = -1, /* okapi IllegalArgumentException */
  CAPF_ERR_NOT_IMPLEMENTED = -2,  /* okapi NotImplementedException   */
  CAPF_ERR_INTERNAL = -3,         /* okapi IllegalStateException / InternalException */
  CAPF_ERR_HIP = -4,              /* HIP runtime failure               */
  CAPF_ERR_OOM = -5               /* device allocation failed          */
};

/* column types (FlinkConversions.scala:43-117) */
enum {
  CAPF_TYPE_NULL = 0,    /* CTNull: column of nulls */
  CAPF_TYPE_INT64 = 1,   /* CTInteger, CTNode/CTRelationship/CTIdentity ids (Types.LONG) */
  CAPF_TYPE_FLOAT64 = 2, /* CTFloat (Types.DOUBLE) */
  CAPF_TYPE_BOOL = 3,    /* CTBoolean, HasLabel / HasType columns */
  CAPF_TYPE_STRING = 4,  /* CTString, stored as int64 dictionary codes */
  CAPF_TYPE_LIST = 5     /* CTList(elem): the result of collect (see capf_table_list_info) */
};

/* join types (okapi-relational/.../impl/planning/PhysicalConstants.scala:29-35) */
enum {
  CAPF_JOIN_INNER = 0,
  CAPF_JOIN_LEFT_OUTER = 1,
  CAPF_JOIN_RIGHT_OUTER = 2,
  CAPF_JOIN_FULL_OUTER = 3,
  CAPF_JOIN_CROSS = 4
};

/* aggregators (okapi-ir/.../api/expr/Expr.scala:1031-1140,
 * lowered as in FlinkSQLExprMapper.scala:281-287) */
enum {
  CAPF_AGG_COUNT_STAR = 0,
  CAPF_AGG_COUNT = 1,
  CAPF_AGG_SUM = 2,
  CAPF_AGG_MIN = 3,
  CAPF_AGG_MAX = 4,
  CAPF_AGG_AVG = 5,
  /* Collect (Expr.scala Collect; Flink child0.collect, FlinkSQLExprMapper.scala:283):
   * the non-NULL values of each group as a LIST column (empty list for none);
   * agg_distinct drops duplicate values.  Flink's COLLECT is a MULTISET: the
   * element order is not part of the result (here: ascending values, string
   * elements in dictionary-code order). */
  CAPF_AGG_COLLECT = 6,
  /* StDev / StDevP (Expr.scala:1120-1128; Flink child0.stddevSamp / stddevPop,
   * FlinkSQLExprMapper.scala:223-224): the sample / population standard
   * deviation of the group's non-NULL numeric values as a FLOAT; NULL for a
   * group without values (AggregationTests.scala:610-617, 637-644) and, for
   * the sample form, with one value (Calcite's STDDEV_SAMP divides by
   * count - 1 and yields NULL for count = 1).  Two-pass, double-double sums. */
  CAPF_AGG_STDEV = 7,
  CAPF_AGG_STDEV_POP = 8,
  /* PercentileCont / PercentileDisc (Expr.scala:1096-1118) with the fraction
   * p = agg_params[i] in [0, 1] of capf_table_group_ex.  The semantics of the
   * Spark backend of the same SPI (morpheus-spark-cypher/.../impl/expressions/
   * PercentileUdafs.scala:59-96; Flink has no mapping): over the sorted
   * non-NULL values v[0..n), disc = v[max(round(n·p), 1) − 1] in the input's
   * type; cont = linear interpolation at position 1 + (n − 1)·p, a FLOAT.
   * NULL for a group without values.                                        */
  CAPF_AGG_PERCENTILE_CONT = 9,
  CAPF_AGG_PERCENTILE_DISC = 10
};

/*
 * Expression programs.  The shim lowers the supported subset of okapi `Expr`
 * trees (what FlinkSQLExprMapper.asFlinkSQLExpr handles,
 * flink-cypher/.../impl/FlinkSQLExprMapper.scala:48-294) into a postfix
 * program evaluated per row on the GPU with Cypher three-valued logic.
 * Parameters (`Param`) are substituted as literals by the shim.
 */
enum {
  CAPF_OP_COL = 1,         /* push column names[iarg]                       */
  CAPF_OP_LIT_INT = 2,     /* push int64 iarg                               */
  CAPF_OP_LIT_FLOAT = 3,   /* push double farg                              */
  CAPF_OP_LIT_BOOL = 4,    /* push bool iarg != 0                           */
  CAPF_OP_LIT_STRING = 5,  /* push string code iarg (capf_string_intern)    */
  CAPF_OP_LIT_NULL = 6,    /* push NULL of capf type iarg                   */
  CAPF_OP_EQ = 10,         /* Equals            (===)                       */
  CAPF_OP_NEQ = 11,        /* Not(Equals)       fused                       */
  CAPF_OP_LT = 12,         /* LessThan                                      */
  CAPF_OP_LE = 13,         /* LessThanOrEqual                               */
  CAPF_OP_GT = 14,         /* GreaterThan                                   */
  CAPF_OP_GE = 15,         /* GreaterThanOrEqual                            */
  CAPF_OP_NOT = 20,        /* Not                                           */
  CAPF_OP_AND = 21,        /* Ands, arity iarg                              */
  CAPF_OP_OR = 22,         /* Ors,  arity iarg                              */
  CAPF_OP_IS_NULL = 23,    /* IsNull                                        */
  CAPF_OP_IS_NOT_NULL = 24,/* IsNotNull / Exists                            */
  CAPF_OP_ADD = 30,        /* Add (numeric)                                 */
  CAPF_OP_SUB = 31,        /* Subtract                                      */
  CAPF_OP_MUL = 32,        /* Multiply                                      */
  CAPF_OP_DIV = 33,        /* Divide (integer division on int64 operands)   */
  CAPF_OP_MOD = 34,        /* Modulo                                        */
  CAPF_OP_NEG = 35,        /* unary minus                                   */
  CAPF_OP_TO_FLOAT = 40,   /* ToFloat  → DOUBLE                             */
  CAPF_OP_TO_INTEGER = 41, /* ToInteger → Flink casts to INT (32-bit!)      */
  CAPF_OP_COALESCE = 50,   /* Coalesce, arity iarg                          */
  CAPF_OP_STR_LEN = 60,    /* Size(string): pop a STRING, push its length in
                              UTF-16 units (Java String.length, Flink
                              charLength, FlinkSQLExprMapper.scala:80-85)   */
  CAPF_OP_LIST_SIZE = 61,  /* Size(list): push the element count of LIST
                              column names[iarg] (Flink cardinality, :80-85) */
  CAPF_OP_IF = 62,         /* pop value, cond, else: push cond TRUE ? value :
                              else (type(r) over the HasType columns,
                              FlinkSQLExprMapper.scala:152-160; CaseExpr
                              as a chain of Ifs, :242-260); numeric branches
                              of different types widen to FLOAT             */
  /* Mathematical functions (FlinkSQLExprMapper.scala:199-221).  Unary: pop x,
   * push f(x); NULL in, NULL out.  ROUND rounds half away from zero and
   * yields a FLOAT (the Spark mapping round(x).cast(Double),
   * SparkSQLExprMapper.scala:286; Flink's is `???`); CEIL / FLOOR yield
   * FLOAT for FLOAT input, INTEGER input unchanged; SIGN an INTEGER; ABS
   * keeps the type; the rest FLOAT (Java Math.* over doubles).               */
  CAPF_OP_ROUND = 70,
  CAPF_OP_ABS = 71,
  CAPF_OP_CEIL = 72,
  CAPF_OP_FLOOR = 73,
  CAPF_OP_SIGN = 74,
  CAPF_OP_SQRT = 75,
  CAPF_OP_LOG = 76,
  CAPF_OP_LOG10 = 77,
  CAPF_OP_EXP = 78,
  CAPF_OP_SIN = 79,
  CAPF_OP_COS = 80,
  CAPF_OP_TAN = 81,
  CAPF_OP_ASIN = 82,
  CAPF_OP_ACOS = 83,
  CAPF_OP_ATAN = 84,
  CAPF_OP_DEGREES = 85,
  CAPF_OP_RADIANS = 86,
  CAPF_OP_ATAN2 = 87,      /* binary: pop x, y; push atan2(y, x)             */
  /* ToBoolean (:185, Flink cast to BOOLEAN): BOOLEAN unchanged, STRING
   * 'true' / 'false' (any case, trimmed) → TRUE / FALSE, any other string
   * → NULL.  Uses the session's device table of string → boolean codes.     */
  CAPF_OP_TO_BOOLEAN = 88,
  /* x IN [list] over a long INTEGER / STRING list (FlinkSQLExprMapper.scala:
   * 114-118 lowers IN to Flink's `in`): pops x; pushes TRUE when x is in the
   * session literal set names[i] (capf_session_literal_set, referenced as
   * "\x01set:<id>"), else NULL when x is NULL or farg != 0 (the list held a
   * NULL), else FALSE.  One binary search per row over the sorted set.       */
  CAPF_OP_IN_SET = 89,
  /* String functions of one STRING operand and literal arguments (toUpper /
   * toLower / trim / lTrim / rTrim / substring / replace / concatenation with
   * a literal, FlinkSQLExprMapper.scala:120-128, 187-195): pops a STRING code
   * c; pushes entry c of the code map names[iarg] — the function applied to
   * dictionary string c by the caller and interned (capf_session_code_map,
   * referenced as "\x01map:<id>"); NULL in, an entry < 0 (a NULL result) or
   * c past the map → NULL.                                                   */
  CAPF_OP_STR_MAP = 90,
  /* A new STRING per value (toString of an INTEGER / FLOAT column, the
   * concatenation of two columns, :120-128, :184): pops x (farg == 0) or
   * y then x (farg != 0); pushes the code of the value map names[iarg] entry
   * whose key is x's value (INTEGER / STRING code) or bit pattern (FLOAT), or
   * the key pair (x, y); NULL in or no entry → NULL.  The caller evaluated the
   * operands' distinct values, built their strings and interned them
   * (capf_session_value_map, "\x01vmap:<id>").                                */
  CAPF_OP_VALUE_MAP = 91,
  /* toFloat / toInteger of a STRING (FlinkSQLExprMapper.scala:182-183, CAST
   * to DOUBLE / INT): pops a STRING code; iarg 1 pushes it parsed as a
   * DOUBLE (Java Double.valueOf grammar after trim: decimal / exponent forms,
   * NaN, Infinity, an f / d suffix), iarg 0 as an INTEGER (a decimal integer,
   * a fractional part truncated, within 32 bits).  An unparsable string (or
   * NULL) pushes NULL.  Uses the session's device table of parsed strings.   */
  CAPF_OP_STR_TO_NUM = 92,
  /* rand() (:207): pushes a uniform DOUBLE in [0, 1) — splitmix64 of
   * (iarg seed, row); the caller draws a fresh seed per evaluation.          */
  CAPF_OP_RAND = 93,
  /* xs[i] on a LIST column (ContainerIndex, :262-269): pops an INTEGER i;
   * pushes element i of the row's list in LIST column names[iarg] (i < 0
   * counts from the end); NULL for a NULL list, a NULL index or an index out
   * of range.  farg = the element's capf type (CAPF_TYPE_*).                 */
  CAPF_OP_LIST_INDEX = 94,
  /* Ordering of strings (Flink compares VARCHARs lexicographically, Java
   * String.compareTo; FlinkSQLExprMapper.scala:91-94 and ORDER BY): pops a
   * STRING; pushes its INTEGER rank among the session's strings in UTF-16
   * code-unit order, so <, <=, >, >= and sorting on ranks order the strings.
   * NULL in, NULL out.  capf_table_order_by applies it to a STRING key itself. */
  CAPF_OP_STR_RANK = 95
};

typedef struct capf_expr {
  int32_t n;                 /* number of instructions                     */
  const int32_t *ops;        /* opcode per instruction                     */
  const int64_t *iargs;      /* integer immediate per instruction          */
  const double *fargs;       /* float immediate per instruction (may be 0) */
  int32_t n_names;           /* column names referenced by CAPF_OP_COL     */
  const char *const *names;
} capf_expr;

/* ---------------------------------------------------------------- errors */
const char *capf_last_error(void);
int32_t capf_last_error_kind(void);
int32_t capf_abi_version(void);

/* --------------------------------------------------------------- session
 * RelationalCypherSession[T] backend state
 * (okapi-relational/.../api/graph/RelationalCypherSession.scala:63-111;
 *  CAPFSession.create, flink-cypher/.../api/CAPFSession.scala:74-91).
 * `hip_stream` may be NULL (the session creates its own stream) or a
 * hipStream_t owned by the caller (e.g. torch.cuda.current_stream()).     */
capf_status capf_session_create(int32_t device, void *hip_stream, capf_session **out);
capf_status capf_session_destroy(capf_session *s);
capf_status capf_session_sync(capf_session *s);
/* Per-kernel HIP-event timing of the hot kernels (off by default).  reset also
 * sets the last plan back to "none". */
capf_status capf_session_set_profiling(capf_session *s, int32_t enabled);
capf_status capf_session_reset_profile(capf_session *s);
capf_status capf_session_profile_count(capf_session *s, int32_t *n);
capf_status capf_session_profile_entry(capf_session *s, int32_t i, const char **kernel,
                                       int64_t *launches, double *total_ms, double *bytes);
/* last fused execution path taken ("fused_chain2", "fused_triangle", "message_passing",
 * "fused_var_length_reach"; "none" until one runs) */
const char *capf_session_last_plan(capf_session *s);

/* String dictionary for CAPF_TYPE_STRING columns. */
capf_status capf_string_intern(capf_session *s, const char *str, int64_t *code);
capf_status capf_string_lookup(capf_session *s, int64_t code, const char **str);
/* Size and FNV-1a digest of the dictionary in code order: ranks that exchange
 * STRING columns as codes check that their dictionaries agree (dist_table.py). */
capf_status capf_string_digest(capf_session *s, int64_t *count, uint64_t *digest);

/* ---------------------------------------------------- table construction
 * CAPFElementTable.create / CAPFRecordsFactory.from
 * (flink-cypher/.../api/io/CAPFTable.scala:76-83, impl/CAPFRecords.scala:47-100).
 * data[i]: nrows values of 8 bytes (INT64/FLOAT64/STRING) or 1 byte (BOOL),
 *          NULL for a CAPF_TYPE_NULL column.
 * valid[i]: NULL (no nulls) or nrows bytes, 1 = value present.            */
capf_status capf_table_from_host(capf_session *s, int32_t ncols, const char *const *names,
                                 const int32_t *types, const void *const *data,
                                 const uint8_t *const *valid, int64_t nrows, capf_table **out);
/* Same with device pointers; copy = 0 borrows them (caller keeps them alive). */
capf_status capf_table_from_device(capf_session *s, int32_t ncols, const char *const *names,
                                   const int32_t *types, void *const *data,
                                   uint8_t *const *valid, int64_t nrows, int32_t copy,
                                   capf_table **out);
/* RelationalCypherRecordsFactory.unit / empty(header)
 * (okapi-relational/.../api/table/RelationalCypherRecords.scala:43-54)       */
capf_status capf_table_unit(capf_session *s, capf_table **out);
capf_status capf_table_empty(capf_session *s, int32_t ncols, const char *const *names,
                             const int32_t *types, capf_table **out);
capf_status capf_table_retain(capf_table *t);
capf_status capf_table_release(capf_table *t);

/* ------------------------------------------------------------ CypherTable */
/* physicalColumns (CypherTable.scala:48) */
capf_status capf_table_num_columns(capf_table *t, int32_t *n);
capf_status capf_table_column_name(capf_table *t, int32_t i, const char **name);
/* physicalColumns in one call: *joined points at *bytes bytes holding the
 * *n column names, each terminated by '\0' (valid while the table lives)   */
capf_status capf_table_columns(capf_table *t, const char **joined, int64_t *bytes, int32_t *n);
/* columnType (CypherTable.scala:58) */
capf_status capf_table_column_type(capf_table *t, const char *col, int32_t *type);
/* size (CypherTable.scala:68): triggers execution */
capf_status capf_table_size(capf_table *t, int64_t *n);
/* size / group(∅, {count(*)}) without the host wait: the count lands in the
 * device int64 at d_count, ordered on the session stream.  Same value as
 * capf_table_size (CypherTable.scala:68) / the count(*) column of
 * Table.group (Table.scala:158-159); lets a driver plan query i+1 while the
 * GPU runs query i.  Shapes that are not a fused count fall back to the
 * synchronous count (then copy it to d_count).                             */
capf_status capf_table_count_async(capf_table *t, int64_t *d_count);
/* rows (CypherTable.scala:63): download one column; values buffer holds
 * size × (8 or 1) bytes, valid_out (may be NULL) size bytes.              */
capf_status capf_table_download(capf_table *t, const char *col, void *values_out,
                                uint8_t *valid_out);
/* LIST columns (CAPF_TYPE_LIST, from CAPF_AGG_COLLECT).  capf_table_list_info:
 * the element type (CAPF_TYPE_*) and the total element count of column col
 * (n_values NULL: the type alone, read off the plan without evaluating the
 * table whenever the plan determines it — collect, a list literal, labels /
 * keys, or a column passed through select / filter / join / union / sort).
 * capf_table_download_list: offsets_out[size + 1] (int64, list i = elements
 * [offsets[i], offsets[i+1])), values_out[n_values] elements (8 or 1 bytes
 * each, never NULL), valid_out[size] list validity (may be NULL).
 * capf_table_download of a LIST column is CAPF_ERR_ILLEGAL_ARGUMENT.        */
capf_status capf_table_list_info(capf_table *t, const char *col, int32_t *elem_type,
                                 int64_t *n_values);
capf_status capf_table_download_list(capf_table *t, const char *col, int64_t *offsets_out,
                                     void *values_out, uint8_t *valid_out);
/* Device view of a materialised column (for zero-copy interop). */
capf_status capf_table_device_column(capf_table *t, const char *col, void **values,
                                     uint8_t **valid, int64_t *nrows);

/* Storage encodings of a materialised column.  CAPF_ENC_FOR32: INTEGER values
 * held as uint32 offsets from a per-column base (frame of reference) — same
 * values, half the HBM bytes.  No reference counterpart: the Flink backend
 * stores ids as Java longs (CAPFGraph.scala ids are LongType).              */
#define CAPF_ENC_PLAIN 0
#define CAPF_ENC_FOR32 1
#define CAPF_ENC_FOR24 2 /* 3-byte offsets (range < 2^24): 3 B per id */
/* Materialise t and re-encode every INTEGER column whose value range spans
 * < 2^32 as FOR32.  Results of every operator are unchanged.               */
capf_status capf_table_compact(capf_table *t, capf_table **out);
/* The same with a narrowest width: 3 = FOR24 where the range spans < 2^24
 * (FOR32 where it only fits 32 bits), 4 = capf_table_compact.             */
capf_status capf_table_compact_width(capf_table *t, int32_t width, capf_table **out);
capf_status capf_table_column_encoding(capf_table *t, const char *col, int32_t *enc,
                                       int64_t *base);

/* --------------------------------------------------------------- Table[T] */
/* cache() (Table.scala:52) */
capf_status capf_table_cache(capf_table *t, capf_table **out);
/* Not an SPI method: evaluates the lazy operator DAG of t into device
 * memory (what rows / size do before their download or count) — the
 * materialising path timed by bench.py --query one_hop_rows.               */
capf_status capf_table_materialize(capf_table *t);
/* select((col, alias)+) (Table.scala:71) */
capf_status capf_table_select(capf_table *t, int32_t n, const char *const *cols,
                              const char *const *aliases, capf_table **out);
/* filter(expr)(header, params) (Table.scala:81) */
capf_status capf_table_filter(capf_table *t, const capf_expr *pred, capf_table **out);
/* drop(cols*) (Table.scala:89) */
capf_status capf_table_drop(capf_table *t, int32_t n, const char *const *cols, capf_table **out);
/* join(other, joinType, (l, r)*) (Table.scala:99) */
capf_status capf_table_join(capf_table *l, capf_table *r, int32_t join_type, int32_t npairs,
                            const char *const *lcols, const char *const *rcols,
                            capf_table **out);
/* unionAll(other) (Table.scala:107) */
capf_status capf_table_union_all(capf_table *l, capf_table *r, capf_table **out);
/* orderBy((expr, order)*) (Table.scala:115) */
capf_status capf_table_order_by(capf_table *t, int32_t n, const capf_expr *keys,
                                const int32_t *descending, capf_table **out);
/* skip(n) / limit(n) (Table.scala:123, :131) */
capf_status capf_table_skip(capf_table *t, int64_t n, capf_table **out);
capf_status capf_table_limit(capf_table *t, int64_t n, capf_table **out);
/* distinct / distinct(cols*) (Table.scala:138, :146) */
capf_status capf_table_distinct(capf_table *t, capf_table **out);
capf_status capf_table_distinct_cols(capf_table *t, int32_t n, const char *const *cols,
                                     capf_table **out);
/* group(by, aggregations)(header, params) (Table.scala:158-159).
 * by_cols are the physical columns owned by the grouping vars
 * (header.ownedBy, FlinkTable.scala:129-135).                              */
capf_status capf_table_group(capf_table *t, int32_t n_by, const char *const *by_cols,
                             int32_t n_aggs, const int32_t *agg_kinds,
                             const capf_expr *agg_args, const int32_t *agg_distinct,
                             const char *const *agg_names, capf_table **out);
/* group with per-aggregator parameters: agg_params[i] is the percentile
 * fraction of CAPF_AGG_PERCENTILE_CONT / _DISC (ignored for the others; may
 * be NULL when no percentile is requested).  capf_table_group is this call
 * with agg_params = NULL.                                                  */
capf_status capf_table_group_ex(capf_table *t, int32_t n_by, const char *const *by_cols,
                                int32_t n_aggs, const int32_t *agg_kinds,
                                const capf_expr *agg_args, const int32_t *agg_distinct,
                                const double *agg_params, const char *const *agg_names,
                                capf_table **out);
/* withColumns((expr, col)*)(header, params) (Table.scala:170) */
capf_status capf_table_with_columns(capf_table *t, int32_t n, const capf_expr *exprs,
                                    const char *const *names, capf_table **out);
/* UNWIND: withColumns(Explode(list) AS item) (RelationalPlanner.scala:99-101,
 * Explode = FlinkSQLExprMapper.scala:101; row semantics of Spark's explode,
 * SparkSQLExprMapper.scala:146-149): every row of t is repeated once per
 * element of the list, the new column `name` holding the element (rows in
 * input order, elements in list order; an empty list drops the row).
 * capf_table_explode_values: the same literal / parameter list for every row:
 *   n elements of capf type `type` (INT64 / FLOAT64 / BOOL / STRING codes /
 *   NULL), values n × (8 or 1) bytes (NULL for a NULL-typed list), valid
 *   NULL (no NULL elements) or n bytes.
 * capf_table_explode_list: the elements of LIST column list_col (a NULL list
 *   drops the row, like an empty one).  Lazy like every other operator: t is
 *   evaluated with the result, unless list_col is a computed list expression
 *   (its element type is then only known once it exists).                  */
capf_status capf_table_explode_values(capf_table *t, const char *name, int32_t type, int64_t n,
                                      const void *values, const uint8_t *valid, capf_table **out);
capf_status capf_table_explode_list(capf_table *t, const char *list_col, const char *name,
                                    capf_table **out);
/* show(n) (Table.scala:177): prints to stdout */
capf_status capf_table_show(capf_table *t, int32_t rows);

/* ------------------------------------------------ synthetic graph inputs
 * Deterministic Graph500-style R-MAT generator (counter-based, identical to
 * oracle/rmat.c) writing straight into HBM.  Not part of the Table SPI:
 * it stands in for the graph-ingest step (EdgeListDataSource,
 * flink-cypher/.../api/io/edgelist/EdgeListDataSource.scala:56-92).
 * thresholds = floor(a*2^32), floor((a+b)*2^32), floor((a+b+c)*2^32).
 * Produces a relationship table with columns (id_col, src_col, dst_col),
 * rel ids = id_base + edge index, for edges [first, first+count).          */
capf_status capf_rmat_rel_table(capf_session *s, int32_t scale, uint64_t seed,
                                uint32_t t_a, uint32_t t_ab, uint32_t t_abc,
                                int64_t first, int64_t count, int64_t id_base,
                                const char *id_col, const char *src_col,
                                const char *dst_col, capf_table **out);
/* Node table with id column [base, base+n) and an optional BOOL label column
 * label_col (NULL = none) set with probability 1/2 from the seeded hash.  */
capf_status capf_range_node_table(capf_session *s, int64_t base, int64_t n, uint64_t seed,
                                  const char *id_col, const char *label_col,
                                  capf_table **out);

/* ------------------------------------------------------ edge-list ingest
 * EdgeListDataSource.graph (flink-cypher/.../api/io/edgelist/EdgeListDataSource.scala:61-81):
 * a CSV of two LONG fields per line (start, end), field delimiter `sep`
 * (option "sep"), lines beginning with `comment` (option "comment", may be
 * NULL) skipped — CsvTableSource.builder().field(.., LONG) ×2
 * .fieldDelimiter(sep).commentPrefix(comment) (:62-68).  Parsed on the GPU
 * into a relationship table (id_col, src_col, dst_col); ids are the data-line
 * ordinals 0..M-1, one valid zipWithUniqueId assignment (safeAddIdColumn,
 * flink-cypher/.../impl/TableOps.scala:217-238).  A malformed line fails the
 * call with CAPF_ERR_ILLEGAL_ARGUMENT naming the line (Flink: ParseException).
 * capf_edge_list_parse takes the file's bytes; capf_edge_list_read the path. */
capf_status capf_edge_list_parse(capf_session *s, const char *bytes, int64_t nbytes,
                                 const char *sep, const char *comment, const char *id_col,
                                 const char *src_col, const char *dst_col, capf_table **out);
capf_status capf_edge_list_read(capf_session *s, const char *path, const char *sep,
                                const char *comment, const char *id_col, const char *src_col,
                                const char *dst_col, capf_table **out);

/* ----------------------------------------- fused var-length reach (config 5)
 * The fused form of
 *   VarLengthExpand(a, [r*lower..upper], b)   VarLengthExpandPlanner.scala:82-259
 *   → Distinct(a, b)                          FlinkTable.scala:189-196
 *   → Aggregate(by a, count(*) AS reach)      FlinkTable.scala:123-150
 * over a directed relationship scan `rels` (src_col → dst_col), the source
 * node scan `sources` and the target node scan `targets`: one row
 * (out_source_col = a's id, out_reach_col = #distinct b) per source a that
 * reaches at least one target — the rows the relational plan produces,
 * without materialising the paths.  lower = 1 (rel isomorphism cannot change
 * the distinct pairs) and lower = 0 (the copyElement branch,
 * VarLengthExpandPlanner.scala:180-205: every source also pairs with itself,
 * so every source has a row; source ids unique) are fused; other bounds
 * return CAPF_ERR_NOT_IMPLEMENTED and the caller plans the join chain.     */
capf_status capf_var_length_reach(capf_session *s, capf_table *rels, const char *src_col,
                                  const char *dst_col, capf_table *sources,
                                  const char *source_id_col, capf_table *targets,
                                  const char *target_id_col, int32_t lower, int32_t upper,
                                  const char *out_source_col, const char *out_reach_col,
                                  capf_table **out);

/* ------------------------------------------------ multi-GPU partial counts
 * Building blocks of the hash-partitioned 2-hop count: the
 * caller (one process per GPU, torch.distributed/RCCL) exchanges the
 * per-node histograms between ranks.  See DESIGN.md "Multi-GPU".
 * capf_chain2_local_hists: over the rel rows of this rank, writes
 *   in_hist[mix(v - node_base)]  = #rels with dst = v   (v any node)
 *   out_hist[mix(v - node_base)] = #rels with src = v
 * for rels whose endpoints both lie in [node_base, node_base + n_nodes)
 * and returns the number of such self-loops.  Buffers are device uint32
 * arrays of capf_chain2_hist_len(n_nodes) = 2^k >= n_nodes entries, every
 * entry written by the call; mix is the bijection of 2^k node offsets
 * (odd multiply, xorshift; csrc/device_common.h node_mix) the radix
 * partitioning hashes by, so a contiguous 1/G slice of the histogram index
 * is a hash partition of the nodes.                                         */
/* Node-partitioned layout (SURVEY §8(e) "each rel is stored on owner(src);
 * for incoming expansion also a copy on owner(dst)"): owner(v) = the rank
 * whose contiguous range of 64 Ki-index buckets holds mix(v - node_base).
 * capf_table_node_partition: the rows of t whose key_col is owned by `part`
 * of `parts` (the out-copy with key = source, the in-copy with key = target).
 * capf_chain2_sharded_count: this rank's partial of the 2-hop count,
 *   Σ_{b owned} in[b]·out[b] − owned self-loops,
 * in[b] from the in-copy's target column, out[b] from the out-copy's source
 * column (its target column gives the self-loops).  Asynchronous on the
 * session stream; writes the int64 partial to device memory d_partial, ready
 * for one all-reduce (sum) over ranks.  Histograms are session scratch.      */
capf_status capf_table_node_partition(capf_table *t, const char *key_col, int64_t node_base,
                                      int64_t n_nodes, int32_t parts, int32_t part,
                                      capf_table **out);
capf_status capf_chain2_sharded_count(capf_session *s, capf_table *in_copy, const char *in_dst,
                                      capf_table *out_copy, const char *out_src,
                                      const char *out_dst, int64_t node_base, int64_t n_nodes,
                                      int32_t parts, int32_t part, int64_t *d_partial);
/* 2-D layout of the out-copy (a block partition of the adjacency matrix by
 * (owner(source), owner(target)), as distributed graph stores keep it):
 * capf_table_node_partition_diag returns the rows whose source `part` owns
 * with the rows whose target it owns too first (*n_diag of them);
 * capf_chain2_sharded_count_diag is capf_chain2_sharded_count for such an
 * out-copy: a self-loop has both endpoints owned, so the target column is
 * read for rows [0, n_diag) only (n_diag = -1: every row).  hot_ids: up to
 * 2 heavy-hitter node ids (host array; a plan hint sampled at ingest — any
 * ids give the same count): keys equal to one are counted in registers by
 * the partition pass instead of being partitioned (skew handling: a hub's
 * keys would pile onto one LDS counter word in the counting pass).          */
capf_status capf_table_node_partition_diag(capf_table *t, const char *src_col, const char *dst_col,
                                           int64_t node_base, int64_t n_nodes, int32_t parts,
                                           int32_t part, capf_table **out, int64_t *n_diag);
capf_status capf_chain2_sharded_count_diag(capf_session *s, capf_table *in_copy, const char *in_dst,
                                           capf_table *out_copy, const char *out_src,
                                           const char *out_dst, int64_t n_diag, int32_t n_hot,
                                           const int64_t *hot_ids, int64_t node_base,
                                           int64_t n_nodes, int32_t parts, int32_t part,
                                           int64_t *d_partial);
/* Directed triangle (a)-->(b)-->(c)-->(a) with pairwise distinct rels over
 * the rels of `rels` whose endpoints lie in [node_base, node_base + n_nodes)
 * (the fused form of Expand, Expand, ExpandInto + uniqueness,
 * RelationalPlanner.scala:130-189): part `part` of `parts` of the count as a
 * device int64 at d_count — the parts sum to the count (rank r of G computes
 * part r over a replicated rel table, then one all-reduce).  Asynchronous on
 * the session stream after two internal host reads.                         */
capf_status capf_triangle_count_part(capf_session *s, capf_table *rels, const char *src_col,
                                     const char *dst_col, int64_t node_base, int64_t n_nodes,
                                     int32_t parts, int32_t part, int64_t *d_count);
int64_t capf_chain2_hist_len(int64_t n_nodes);
capf_status capf_chain2_local_hists(capf_session *s, capf_table *rels, const char *src_col,
                                    const char *dst_col, int64_t node_base, int64_t n_nodes,
                                    uint32_t *d_in_hist, uint32_t *d_out_hist,
                                    int64_t *self_loops);
/* Σ_v a[v]·b[v] over n entries (device uint32 arrays), exact in uint64. */
capf_status capf_dot_u32(capf_session *s, const uint32_t *d_a, const uint32_t *d_b, int64_t n,
                         uint64_t *out);

/* CSV tables of an FS graph source whose declared fields are all LONG
 * (FSGraphSource.readFromCsv, flink-cypher/.../api/io/fs/FSGraphSource.scala:80-84:
 * Flink's CsvTableSource over the canonical field list of CAPFGraphExport —
 * id, source, target and INTEGER properties).  One INT64 column per declared
 * field, in file order; row rules as capf_edge_list_read (LongParser, trailing
 * '\r' stripped, short rows / empty fields / overflow fail the read naming the
 * line); text after the last declared field is not read.  ncols ≤ 16.      */
capf_status capf_csv_parse_longs(capf_session *s, const char *bytes, int64_t nbytes,
                                 const char *sep, int32_t ncols, const char *const *names,
                                 capf_table **out);
capf_status capf_csv_read_longs(capf_session *s, const char *path, const char *sep,
                                int32_t ncols, const char *const *names, capf_table **out);

/* ------------------------------------------------- distributed Table layer
 * The exchange of a hash-partitioned Table over G ranks (dist_table.py):
 * Flink's join and groupBy repartition both inputs by a hash of the key
 * before the local operator (FlinkTable.scala:171-187 join, :123-150 group
 * lower onto DataSet joinWithTiny/hash-partitioned join and groupBy); here
 * the repartition is this call plus one all-to-all per column (RCCL).
 * capf_table_hash_route: a materialised copy of t whose rows are grouped by
 *   owner = h(values of keys[0..nkeys)) of `parts` (owner order, stable inside
 *   an owner); counts[p] = rows owned by p (host array of `parts`).  Equal key
 *   tuples have equal owners; NULLs of a key route together; −0.0 as 0.0.
 *   LIST columns cannot be routed (CAPF_ERR_ILLEGAL_ARGUMENT).
 * capf_table_download_device: `rows` of one column into DEVICE buffers
 *   (decoded values, size × 8 or 1 bytes; d_valid = size bytes, 1 = present).
 * capf_table_has_nulls: does column col carry a validity array (or is it
 *   an all-NULL column with rows)?                                          */
capf_status capf_table_hash_route(capf_table *t, int32_t nkeys, const char *const *keys,
                                  int32_t parts, int64_t *counts, capf_table **out);
capf_status capf_table_download_device(capf_table *t, const char *col, void *d_values,
                                       uint8_t *d_valid);
capf_status capf_table_has_nulls(capf_table *t, const char *col, int32_t *has);

/* Exchange wire format of the distributed Table layer (dist_table.py: one
 * all_to_all_single per shuffle, Flink's hash repartition in FlinkTable.scala:
 * 123-196).  A row is packed as, per column i: width[i] bytes of
 * (value − base[i]) little-endian — 3 / 4 for INTEGER / STRING columns whose
 * range over every rank fits 24 / 32 bits (FOR24 / FOR32), 8 otherwise and for
 * FLOAT (base 0), 1 for BOOL, 0 for NULL — then one validity byte when
 * nullable[i].  capf_table_column_range: min / max / non-NULL count of an
 * INTEGER or STRING column (column statistics, computed once).
 * capf_table_pack_rows: *row_bytes = W; rows into d_out (n·W device bytes; null
 * d_out: only W).  capf_table_from_packed_rows: the table of nrows packed rows
 * at d_rows (copied out; the narrow widths stay FOR24 / FOR32 encoded).       */
capf_status capf_table_column_range(capf_table *t, const char *col, int64_t *min, int64_t *max,
                                    int64_t *non_null);
capf_status capf_table_pack_rows(capf_table *t, int32_t ncols, const char *const *cols, const int32_t *width,
                                 const int64_t *base, const int32_t *nullable, int32_t *row_bytes, void *d_out);
capf_status capf_table_from_packed_rows(capf_session *s, int32_t ncols, const char *const *names,
                                        const int32_t *types, const int32_t *width, const int64_t *base,
                                        const int32_t *nullable, const void *d_rows, int64_t nrows,
                                        capf_table **out);

/* ------------------------------------------------- rank communicator (RCCL)
 * The exchange of the distributed Table layer for hosts without a framework
 * communicator (the JVM twin DistGpuTable.scala; the Python layer uses
 * torch.distributed for the same collectives): RCCL over xGMI, one process per
 * GPU, every collective enqueued on the session's stream (ordered with the
 * kernels that produce and consume its buffers).  It replaces Flink's hash
 * repartition between operator instances (FlinkTable.scala:123-196).
 * capf_comm_unique_id: rank 0 creates the id (128 bytes) and sends it to the
 *   other ranks out of band; every rank then calls capf_comm_init with it.
 * capf_comm_all_reduce_i64: in place, op CAPF_COMM_SUM / CAPF_COMM_MAX.
 * capf_comm_all_gather_bytes: `bytes` from every rank, rank-major into d_recv
 *   (world × bytes).
 * capf_comm_all_to_all_bytes: send_bytes[p] bytes (consecutive in d_send, rank
 *   order) to rank p, recv_bytes[p] from rank p into d_recv (rank order) —
 *   the packed-row shuffle of capf_table_pack_rows.
 * capf_session_alloc / capf_session_free: device buffers from the session's
 *   stream-ordered pool (exchange buffers, count slots);
 * capf_session_copy: hipMemcpyAsync on the session stream + wait (kind 1 =
 *   host → device, 2 = device → host, 3 = device → device).               */
#define CAPF_COMM_ID_BYTES 128
enum { CAPF_COMM_SUM = 0, CAPF_COMM_MAX = 2 };
typedef struct capf_comm capf_comm;
capf_status capf_comm_unique_id(uint8_t *id_out);
capf_status capf_comm_init(capf_session *s, int32_t world, int32_t rank, const uint8_t *id, capf_comm **out);
capf_status capf_comm_destroy(capf_comm *c);
capf_status capf_comm_rank(capf_comm *c, int32_t *rank, int32_t *world);
capf_status capf_comm_all_reduce_i64(capf_comm *c, int64_t *d_buf, int64_t n, int32_t op);
capf_status capf_comm_all_gather_bytes(capf_comm *c, const void *d_send, int64_t bytes, void *d_recv);
capf_status capf_comm_all_to_all_bytes(capf_comm *c, const void *d_send, const int64_t *send_bytes,
                                       void *d_recv, const int64_t *recv_bytes);
capf_status capf_session_alloc(capf_session *s, int64_t bytes, void **d_out);
capf_status capf_session_free(capf_session *s, void *d);
capf_status capf_session_copy(capf_session *s, void *dst, const void *src, int64_t bytes, int32_t kind);

/* A literal set for CAPF_OP_IN_SET: the n int64 values (INTEGER values or
 * STRING dictionary codes) sorted and deduplicated into device memory owned by
 * the session; *set_id names it in programs as "\x01set:<set_id>".  The same
 * values registered again return the same id. */
capf_status capf_session_literal_set(capf_session *s, const int64_t *values, int64_t n, int32_t *set_id);
/* A code map of CAPF_OP_STR_MAP: codes[c] = the STRING code the function gives
 * dictionary string c (−1: NULL), for c < n.  The caller (the shim) applies the
 * function on the host with the JVM's string semantics and interns the
 * results; the map is referenced in programs as "\x01map:<id>" (*map_id).  */
capf_status capf_session_code_map(capf_session *s, const int64_t *codes, int64_t n, int32_t *map_id);
/* The code map map_id grown to n entries after the dictionary has grown:
 * codes[0 .. old n) must be the map's codes.  Replaced in place (*new_id =
 * map_id; the old table is released once the launches already enqueued have
 * read it, and programs naming the id read the longer map) when this is the
 * map's only registration; otherwise (equal maps registered for several
 * functions) a new map is registered and *new_id names it.               */
capf_status capf_session_code_map_extend(capf_session *s, int32_t map_id, const int64_t *codes, int64_t n,
                                         int32_t *new_id);
/* A LIST property column from host data (CTList properties of element tables,
 * CAPFElementTable.create / FlinkConversions.scala:43-117 map CTList to an
 * ARRAY column): appends LIST column `name` to t's rows (t is materialised):
 * row i holds values[offsets[i] .. offsets[i + 1]) (offsets: size + 1 int64,
 * offsets[0] = 0), elements of capf type elem_type (INTEGER / FLOAT / BOOLEAN
 * / STRING codes, 8 B each, BOOLEAN 1 B; no NULL elements); valid (size
 * bytes or NULL): 0 = a NULL list.                                         */
capf_status capf_table_add_list(capf_table *t, const char *name, int32_t elem_type, const int64_t *offsets,
                                const void *values, const uint8_t *valid, capf_table **out);

/* This table plus LIST column `name` whose row i holds (cols[0][i], ...,
 * cols[n-1][i]) — a list literal of per-row elements, `[n.val * 10, $p]`
 * (replaces FlinkSQLExprMapper.scala:71 `array(...)` over the converted
 * children).  The element columns share one type (INTEGER and FLOAT widen to
 * FLOAT); a NULL-typed or NULL-holding element is NotImplemented (LIST columns
 * hold no NULL elements), as are nested lists.  n = 0: the empty list.       */
capf_status capf_table_list_columns(capf_table *t, int32_t n, const char *const *cols, const char *name,
                                    capf_table **out);
/* labels(n) / keys(n) (FlinkSQLExprMapper.scala:136-153; the GetLabels /
 * GetKeys UDFs, :310-329): appends LIST<STRING> column `name` holding, per row,
 * codes[j] for each column cols[j] that holds TRUE (kinds[j] = 0, a label flag)
 * or any value (kinds[j] = 1, a property), in the given order (the shim sorts
 * by label / key name); never NULL (an empty list).                        */
capf_status capf_table_name_list(capf_table *t, int32_t n, const char *const *cols, const int32_t *kinds,
                                 const int64_t *codes, const char *name, capf_table **out);
/* A value map of CAPF_OP_VALUE_MAP: n keys (keys2 = NULL) or key pairs sorted
 * ascending as signed int64 (pairs lexicographically), codes[i] the STRING code
 * of entry i; referenced as "\x01vmap:<id>" (*map_id).                      */
capf_status capf_session_value_map(capf_session *s, const int64_t *keys, const int64_t *keys2, const int64_t *codes,
                                   int64_t n, int32_t *map_id);

#ifdef __cplusplus
}
#endif
#endif /* CAPF_GPU_H */
