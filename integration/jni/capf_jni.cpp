// capf_jni.cpp — JNI adapter binding EVERY entry point of include/capf_gpu.h
// to `object org.opencypher.gpu.Native` (integration/scala/.../Native.scala),
// the native half of the `GpuTable extends Table[GpuTable]` backend that
// replaces FlinkTable (flink-cypher/.../impl/table/FlinkTable.scala:49-199)
// under the unchanged okapi-relational planner.
//
// Build (on a machine with a JDK; not part of this repo's build, which has no JVM):
//   g++ -O2 -std=c++17 -fPIC -shared -I$JAVA_HOME/include -I$JAVA_HOME/include/linux
//       -I include integration/jni/capf_jni.cpp -L cypher-for-apache-flink_amd -lcapf_gpu
//       -o libcapf_jni.so
// tests/test_jni_shim.py type-checks this file against include/capf_gpu.h with
// g++ -fsyntax-only and a minimal declaration of the JNI types it uses.
//
// Conventions of the binding
//  - capf_session* / capf_table* travel as jlong handles; every table handle a
//    native method returns is owned by the caller (GpuTable registers a
//    Cleaner that calls tableRelease, capf_table_release).
//  - A failing status throws org.opencypher.gpu.CapfNativeException(kind,
//    message) with capf_last_error_kind() / capf_last_error(); Native.scala
//    rethrows it as the okapi exception of that kind
//    (okapi-api/.../impl/exception/InternalException.scala:36-65), as FlinkTable
//    surfaces Flink's exceptions.
//  - Expressions arrive as org.opencypher.gpu.Program objects (fields ops: int[],
//    iargs: long[], fargs: double[], names: String[]) — the postfix form of
//    capf_expr built by GpuExprMapper (the counterpart of
//    FlinkSQLExprMapper.asFlinkSQLExpr, flink-cypher/.../impl/FlinkSQLExprMapper.scala:48-294).
//  - Host column data are direct java.nio.ByteBuffers (no copy through the JVM
//    heap); device pointers (HIP / torch interop) are jlong addresses.
#include <jni.h>

#include <cstdint>
#include <string>
#include <vector>

#include "capf_gpu.h"

namespace {

// ---------------------------------------------------------------- errors
bool fail(JNIEnv *env, capf_status st) {
  if (st == CAPF_OK) return false;
  jclass cls = env->FindClass("org/opencypher/gpu/CapfNativeException");
  if (!cls) return true;  // NoClassDefFoundError already pending
  jmethodID ctor = env->GetMethodID(cls, "<init>", "(ILjava/lang/String;)V");
  const char *msg = capf_last_error();
  jstring jmsg = env->NewStringUTF(msg ? msg : "capf error");
  jobject ex = env->NewObject(cls, ctor, (jint)capf_last_error_kind(), jmsg);
  env->Throw((jthrowable)ex);
  return true;
}

// an IllegalArgumentException (okapi's IllegalArgumentException is thrown by the
// Scala side from it) — for argument arrays whose lengths disagree
bool illegal_argument(JNIEnv *env, const char *msg) {
  jclass cls = env->FindClass("java/lang/IllegalArgumentException");
  if (cls) env->ThrowNew(cls, msg);
  return true;
}

capf_session *S(jlong h) { return reinterpret_cast<capf_session *>(h); }
capf_table *T(jlong h) { return reinterpret_cast<capf_table *>(h); }
jlong H(capf_table *t) { return reinterpret_cast<jlong>(t); }

// ---------------------------------------------------------------- strings
struct JStr {
  JNIEnv *env;
  jstring js;
  const char *p;
  JStr(JNIEnv *e, jstring s) : env(e), js(s), p(s ? e->GetStringUTFChars(s, nullptr) : nullptr) {}
  ~JStr() {
    if (p) env->ReleaseStringUTFChars(js, p);
  }
  JStr(const JStr &) = delete;
  JStr &operator=(const JStr &) = delete;
};

struct JStrs {  // String[] → const char *const *
  std::vector<std::string> own;
  std::vector<const char *> ptr;
  JStrs(JNIEnv *env, jobjectArray a) {
    const jsize n = a ? env->GetArrayLength(a) : 0;
    own.reserve(n);
    for (jsize i = 0; i < n; ++i) {
      jstring s = (jstring)env->GetObjectArrayElement(a, i);
      JStr c(env, s);
      own.emplace_back(c.p ? c.p : "");
      env->DeleteLocalRef(s);
    }
    for (auto &s : own) ptr.push_back(s.c_str());
  }
  int32_t n() const { return (int32_t)own.size(); }
  const char *const *data() const { return ptr.data(); }
};

jobjectArray to_jstrings(JNIEnv *env, const std::vector<std::string> &v) {
  jclass str = env->FindClass("java/lang/String");
  jobjectArray a = env->NewObjectArray((jsize)v.size(), str, nullptr);
  for (size_t i = 0; i < v.size(); ++i) {
    jstring s = env->NewStringUTF(v[i].c_str());
    env->SetObjectArrayElement(a, (jsize)i, s);
    env->DeleteLocalRef(s);
  }
  return a;
}

std::vector<int32_t> ints(JNIEnv *env, jintArray a) {
  std::vector<int32_t> v(a ? env->GetArrayLength(a) : 0);
  if (!v.empty()) env->GetIntArrayRegion(a, 0, (jsize)v.size(), reinterpret_cast<jint *>(v.data()));
  return v;
}
std::vector<int64_t> longs(JNIEnv *env, jlongArray a) {
  std::vector<int64_t> v(a ? env->GetArrayLength(a) : 0);
  if (!v.empty()) env->GetLongArrayRegion(a, 0, (jsize)v.size(), reinterpret_cast<jlong *>(v.data()));
  return v;
}
std::vector<double> doubles(JNIEnv *env, jdoubleArray a) {
  std::vector<double> v(a ? env->GetArrayLength(a) : 0);
  if (!v.empty()) env->GetDoubleArrayRegion(a, 0, (jsize)v.size(), v.data());
  return v;
}
std::vector<int32_t> bools(JNIEnv *env, jbooleanArray a) {
  const jsize n = a ? env->GetArrayLength(a) : 0;
  std::vector<jboolean> b(n);
  if (n) env->GetBooleanArrayRegion(a, 0, n, b.data());
  return std::vector<int32_t>(b.begin(), b.end());
}

// ---------------------------------------------------------------- programs
// org.opencypher.gpu.Program → capf_expr (owns the arrays it points at)
struct Program {
  std::vector<int32_t> ops;
  std::vector<int64_t> iargs;
  std::vector<double> fargs;
  JStrs *names = nullptr;
  capf_expr e{};
  Program(JNIEnv *env, jobject p) {
    jclass cls = env->GetObjectClass(p);
    ops = ints(env, (jintArray)env->GetObjectField(p, env->GetFieldID(cls, "ops", "[I")));
    iargs = longs(env, (jlongArray)env->GetObjectField(p, env->GetFieldID(cls, "iargs", "[J")));
    fargs = doubles(env, (jdoubleArray)env->GetObjectField(p, env->GetFieldID(cls, "fargs", "[D")));
    names = new JStrs(env, (jobjectArray)env->GetObjectField(
                               p, env->GetFieldID(cls, "names", "[Ljava/lang/String;")));
    e.n = (int32_t)ops.size();
    e.ops = ops.data();
    e.iargs = iargs.data();
    e.fargs = fargs.empty() ? nullptr : fargs.data();
    e.n_names = names->n();
    e.names = names->data();
  }
  ~Program() { delete names; }
  Program(const Program &) = delete;
  Program &operator=(const Program &) = delete;
};

struct Programs {  // Program[] → contiguous capf_expr[]
  std::vector<Program *> own;
  std::vector<capf_expr> exprs;
  Programs(JNIEnv *env, jobjectArray a) {
    const jsize n = a ? env->GetArrayLength(a) : 0;
    for (jsize i = 0; i < n; ++i) {
      jobject p = env->GetObjectArrayElement(a, i);
      own.push_back(new Program(env, p));
      exprs.push_back(own.back()->e);
      env->DeleteLocalRef(p);
    }
  }
  ~Programs() {
    for (auto *p : own) delete p;
  }
  int32_t n() const { return (int32_t)exprs.size(); }
  const capf_expr *data() const { return exprs.data(); }
};

void *direct(JNIEnv *env, jobject buf) { return buf ? env->GetDirectBufferAddress(buf) : nullptr; }

}  // namespace

#define JNI(ret, name) extern "C" JNIEXPORT ret JNICALL Java_org_opencypher_gpu_Native_00024_##name
// (Scala `object Native` compiles to class Native$ — hence the _00024 mangling;
//  the methods are instance methods of the singleton: (JNIEnv*, jobject self, ...))

// ---------------------------------------------------------------- errors / ABI
JNI(jstring, lastError)(JNIEnv *env, jobject) {
  const char *m = capf_last_error();
  return env->NewStringUTF(m ? m : "");
}
JNI(jint, lastErrorKind)(JNIEnv *, jobject) { return capf_last_error_kind(); }
JNI(jint, abiVersion)(JNIEnv *, jobject) { return capf_abi_version(); }

// ---------------------------------------------------------------- session
// RelationalCypherSession backend state (RelationalCypherSession.scala:63-111)
JNI(jlong, sessionCreate)(JNIEnv *env, jobject, jint device, jlong hip_stream) {
  capf_session *s = nullptr;
  if (fail(env, capf_session_create(device, reinterpret_cast<void *>(hip_stream), &s))) return 0;
  return reinterpret_cast<jlong>(s);
}
JNI(void, sessionDestroy)(JNIEnv *env, jobject, jlong s) { fail(env, capf_session_destroy(S(s))); }
JNI(void, sessionSync)(JNIEnv *env, jobject, jlong s) { fail(env, capf_session_sync(S(s))); }
JNI(void, sessionSetProfiling)(JNIEnv *env, jobject, jlong s, jboolean on) {
  fail(env, capf_session_set_profiling(S(s), on ? 1 : 0));
}
JNI(void, sessionResetProfile)(JNIEnv *env, jobject, jlong s) {
  fail(env, capf_session_reset_profile(S(s)));
}
JNI(jint, sessionProfileCount)(JNIEnv *env, jobject, jlong s) {
  int32_t n = 0;
  fail(env, capf_session_profile_count(S(s), &n));
  return n;
}
// entry i: returns the kernel name; launches → launchesOut[0], (total_ms, bytes) → msBytesOut
JNI(jstring, sessionProfileEntry)(JNIEnv *env, jobject, jlong s, jint i, jlongArray launchesOut,
                                  jdoubleArray msBytesOut) {
  const char *k = nullptr;
  int64_t launches = 0;
  double ms = 0, bytes = 0;
  if (fail(env, capf_session_profile_entry(S(s), i, &k, &launches, &ms, &bytes))) return nullptr;
  jlong l = launches;
  jdouble mb[2] = {ms, bytes};
  env->SetLongArrayRegion(launchesOut, 0, 1, &l);
  env->SetDoubleArrayRegion(msBytesOut, 0, 2, mb);
  return env->NewStringUTF(k ? k : "");
}
JNI(jstring, sessionLastPlan)(JNIEnv *env, jobject, jlong s) {
  const char *p = capf_session_last_plan(S(s));
  return env->NewStringUTF(p ? p : "");
}

// CTString dictionary
JNI(jlong, stringIntern)(JNIEnv *env, jobject, jlong s, jstring str) {
  JStr c(env, str);
  int64_t code = 0;
  fail(env, capf_string_intern(S(s), c.p, &code));
  return code;
}
JNI(jstring, stringLookup)(JNIEnv *env, jobject, jlong s, jlong code) {
  const char *p = nullptr;
  if (fail(env, capf_string_lookup(S(s), code, &p))) return nullptr;
  return env->NewStringUTF(p ? p : "");
}
// out[0] = dictionary size, out[1] = FNV-1a digest (bits)
JNI(void, stringDigest)(JNIEnv *env, jobject, jlong s, jlongArray out) {
  int64_t n = 0;
  uint64_t d = 0;
  if (fail(env, capf_string_digest(S(s), &n, &d))) return;
  jlong v[2] = {(jlong)n, (jlong)d};
  env->SetLongArrayRegion(out, 0, 2, v);
}

// ---------------------------------------------------------------- construction
// CAPFElementTable.create / CAPFRecordsFactory.from (CAPFTable.scala:76-83,
// CAPFRecords.scala:47-100): columns as direct buffers (8 B or 1 B per row)
JNI(jlong, tableFromHost)(JNIEnv *env, jobject, jlong s, jobjectArray names, jintArray types,
                          jobjectArray data, jobjectArray valid, jlong nrows) {
  JStrs nm(env, names);
  std::vector<int32_t> ty = ints(env, types);
  if ((int32_t)ty.size() != nm.n() || !data || env->GetArrayLength(data) != nm.n() ||
      (valid && env->GetArrayLength(valid) != nm.n())) {
    illegal_argument(env, "tableFromHost: types, data and valid need one entry per column");
    return 0;
  }
  std::vector<const void *> d(nm.n(), nullptr);
  std::vector<const uint8_t *> v(nm.n(), nullptr);
  for (int32_t i = 0; i < nm.n(); ++i) {
    jobject b = env->GetObjectArrayElement(data, i);
    d[i] = direct(env, b);
    if (b) env->DeleteLocalRef(b);
    if (valid) {
      jobject m = env->GetObjectArrayElement(valid, i);
      v[i] = (const uint8_t *)direct(env, m);
      if (m) env->DeleteLocalRef(m);
    }
  }
  capf_table *out = nullptr;
  if (fail(env, capf_table_from_host(S(s), nm.n(), nm.data(), ty.data(), d.data(), v.data(), nrows,
                                     &out)))
    return 0;
  return H(out);
}
JNI(jlong, tableFromDevice)(JNIEnv *env, jobject, jlong s, jobjectArray names, jintArray types,
                            jlongArray data, jlongArray valid, jlong nrows, jboolean copy) {
  JStrs nm(env, names);
  std::vector<int32_t> ty = ints(env, types);
  std::vector<int64_t> dp = longs(env, data), vp = longs(env, valid);
  if ((int32_t)ty.size() != nm.n() || (int32_t)dp.size() != nm.n() || (!vp.empty() && (int32_t)vp.size() != nm.n())) {
    illegal_argument(env, "tableFromDevice: types, data and valid need one entry per column");
    return 0;
  }
  std::vector<void *> d(nm.n(), nullptr);
  std::vector<uint8_t *> v(nm.n(), nullptr);
  for (int32_t i = 0; i < nm.n(); ++i) {
    d[i] = reinterpret_cast<void *>(dp[i]);
    if (!vp.empty()) v[i] = reinterpret_cast<uint8_t *>(vp[i]);
  }
  capf_table *out = nullptr;
  if (fail(env, capf_table_from_device(S(s), nm.n(), nm.data(), ty.data(), d.data(), v.data(),
                                       nrows, copy ? 1 : 0, &out)))
    return 0;
  return H(out);
}
// RelationalCypherRecordsFactory.unit / empty (RelationalCypherRecords.scala:43-54)
JNI(jlong, tableUnit)(JNIEnv *env, jobject, jlong s) {
  capf_table *out = nullptr;
  return fail(env, capf_table_unit(S(s), &out)) ? 0 : H(out);
}
JNI(jlong, tableEmpty)(JNIEnv *env, jobject, jlong s, jobjectArray names, jintArray types) {
  JStrs nm(env, names);
  std::vector<int32_t> ty = ints(env, types);
  capf_table *out = nullptr;
  return fail(env, capf_table_empty(S(s), nm.n(), nm.data(), ty.data(), &out)) ? 0 : H(out);
}
JNI(void, tableRetain)(JNIEnv *env, jobject, jlong t) { fail(env, capf_table_retain(T(t))); }
JNI(void, tableRelease)(JNIEnv *env, jobject, jlong t) { fail(env, capf_table_release(T(t))); }

// ---------------------------------------------------------------- CypherTable
// physicalColumns (CypherTable.scala:48)
JNI(jobjectArray, tableColumns)(JNIEnv *env, jobject, jlong t) {
  const char *joined = nullptr;
  int64_t bytes = 0;
  int32_t n = 0;
  if (fail(env, capf_table_columns(T(t), &joined, &bytes, &n))) return nullptr;
  std::vector<std::string> cols;
  const char *p = joined;
  for (int32_t i = 0; i < n; ++i) {
    cols.emplace_back(p);
    p += cols.back().size() + 1;
  }
  return to_jstrings(env, cols);
}
JNI(jint, tableNumColumns)(JNIEnv *env, jobject, jlong t) {
  int32_t n = 0;
  fail(env, capf_table_num_columns(T(t), &n));
  return n;
}
JNI(jstring, tableColumnName)(JNIEnv *env, jobject, jlong t, jint i) {
  const char *p = nullptr;
  if (fail(env, capf_table_column_name(T(t), i, &p))) return nullptr;
  return env->NewStringUTF(p);
}
// columnType (CypherTable.scala:58)
JNI(jint, tableColumnType)(JNIEnv *env, jobject, jlong t, jstring col) {
  JStr c(env, col);
  int32_t ty = 0;
  fail(env, capf_table_column_type(T(t), c.p, &ty));
  return ty;
}
// size (CypherTable.scala:68)
JNI(jlong, tableSize)(JNIEnv *env, jobject, jlong t) {
  int64_t n = 0;
  fail(env, capf_table_size(T(t), &n));
  return n;
}
JNI(void, tableCountAsync)(JNIEnv *env, jobject, jlong t, jlong d_count) {
  fail(env, capf_table_count_async(T(t), reinterpret_cast<int64_t *>(d_count)));
}
// rows (CypherTable.scala:63): one column into direct buffers
JNI(void, tableDownload)(JNIEnv *env, jobject, jlong t, jstring col, jobject values,
                         jobject valid) {
  JStr c(env, col);
  fail(env, capf_table_download(T(t), c.p, direct(env, values), (uint8_t *)direct(env, valid)));
}
// LIST columns (collect): returns the element type; element count → nValuesOut[0]
// (nValuesOut null: the type alone, read off the plan without evaluating it)
JNI(jint, tableListInfo)(JNIEnv *env, jobject, jlong t, jstring col, jlongArray nValuesOut) {
  JStr c(env, col);
  int32_t elem = 0;
  int64_t nv = 0;
  if (fail(env, capf_table_list_info(T(t), c.p, &elem, nValuesOut ? &nv : nullptr))) return 0;
  if (nValuesOut) {
    jlong v = nv;
    env->SetLongArrayRegion(nValuesOut, 0, 1, &v);
  }
  return elem;
}
JNI(void, tableDownloadList)(JNIEnv *env, jobject, jlong t, jstring col, jobject offsets,
                             jobject values, jobject valid) {
  JStr c(env, col);
  fail(env, capf_table_download_list(T(t), c.p, (int64_t *)direct(env, offsets), direct(env, values),
                                     (uint8_t *)direct(env, valid)));
}
// device view: out = {values, valid, nrows}
JNI(void, tableDeviceColumn)(JNIEnv *env, jobject, jlong t, jstring col, jlongArray out) {
  JStr c(env, col);
  void *values = nullptr;
  uint8_t *valid = nullptr;
  int64_t n = 0;
  if (fail(env, capf_table_device_column(T(t), c.p, &values, &valid, &n))) return;
  jlong r[3] = {reinterpret_cast<jlong>(values), reinterpret_cast<jlong>(valid), n};
  env->SetLongArrayRegion(out, 0, 3, r);
}
JNI(jlong, tableCompact)(JNIEnv *env, jobject, jlong t) {
  capf_table *out = nullptr;
  return fail(env, capf_table_compact(T(t), &out)) ? 0 : H(out);
}
JNI(jlong, tableCompactWidth)(JNIEnv *env, jobject, jlong t, jint width) {
  capf_table *out = nullptr;
  return fail(env, capf_table_compact_width(T(t), width, &out)) ? 0 : H(out);
}
// returns the encoding; base → baseOut[0]
JNI(jint, tableColumnEncoding)(JNIEnv *env, jobject, jlong t, jstring col, jlongArray baseOut) {
  JStr c(env, col);
  int32_t enc = 0;
  int64_t base = 0;
  if (fail(env, capf_table_column_encoding(T(t), c.p, &enc, &base))) return 0;
  jlong b = base;
  env->SetLongArrayRegion(baseOut, 0, 1, &b);
  return enc;
}

// ---------------------------------------------------------------- Table[T]
JNI(jlong, tableCache)(JNIEnv *env, jobject, jlong t) {  // Table.scala:52
  capf_table *out = nullptr;
  return fail(env, capf_table_cache(T(t), &out)) ? 0 : H(out);
}
JNI(void, tableMaterialize)(JNIEnv *env, jobject, jlong t) {
  fail(env, capf_table_materialize(T(t)));
}
JNI(jlong, tableSelect)(JNIEnv *env, jobject, jlong t, jobjectArray cols,
                        jobjectArray aliases) {  // Table.scala:71
  JStrs c(env, cols), a(env, aliases);
  capf_table *out = nullptr;
  return fail(env, capf_table_select(T(t), c.n(), c.data(), a.data(), &out)) ? 0 : H(out);
}
JNI(jlong, tableFilter)(JNIEnv *env, jobject, jlong t, jobject pred) {  // Table.scala:81
  Program p(env, pred);
  capf_table *out = nullptr;
  return fail(env, capf_table_filter(T(t), &p.e, &out)) ? 0 : H(out);
}
JNI(jlong, tableDrop)(JNIEnv *env, jobject, jlong t, jobjectArray cols) {  // Table.scala:89
  JStrs c(env, cols);
  capf_table *out = nullptr;
  return fail(env, capf_table_drop(T(t), c.n(), c.data(), &out)) ? 0 : H(out);
}
JNI(jlong, tableJoin)(JNIEnv *env, jobject, jlong l, jlong r, jint join_type, jobjectArray lcols,
                      jobjectArray rcols) {  // Table.scala:99
  JStrs lc(env, lcols), rc(env, rcols);
  capf_table *out = nullptr;
  return fail(env, capf_table_join(T(l), T(r), join_type, lc.n(), lc.data(), rc.data(), &out))
             ? 0
             : H(out);
}
JNI(jlong, tableUnionAll)(JNIEnv *env, jobject, jlong l, jlong r) {  // Table.scala:107
  capf_table *out = nullptr;
  return fail(env, capf_table_union_all(T(l), T(r), &out)) ? 0 : H(out);
}
JNI(jlong, tableOrderBy)(JNIEnv *env, jobject, jlong t, jobjectArray keys,
                         jbooleanArray descending) {  // Table.scala:115
  Programs k(env, keys);
  std::vector<int32_t> d = bools(env, descending);
  capf_table *out = nullptr;
  return fail(env, capf_table_order_by(T(t), k.n(), k.data(), d.data(), &out)) ? 0 : H(out);
}
JNI(jlong, tableSkip)(JNIEnv *env, jobject, jlong t, jlong n) {  // Table.scala:123
  capf_table *out = nullptr;
  return fail(env, capf_table_skip(T(t), n, &out)) ? 0 : H(out);
}
JNI(jlong, tableLimit)(JNIEnv *env, jobject, jlong t, jlong n) {  // Table.scala:131
  capf_table *out = nullptr;
  return fail(env, capf_table_limit(T(t), n, &out)) ? 0 : H(out);
}
JNI(jlong, tableDistinct)(JNIEnv *env, jobject, jlong t) {  // Table.scala:138
  capf_table *out = nullptr;
  return fail(env, capf_table_distinct(T(t), &out)) ? 0 : H(out);
}
JNI(jlong, tableDistinctCols)(JNIEnv *env, jobject, jlong t, jobjectArray cols) {  // :146
  JStrs c(env, cols);
  capf_table *out = nullptr;
  return fail(env, capf_table_distinct_cols(T(t), c.n(), c.data(), &out)) ? 0 : H(out);
}
// group(by, aggregations) (Table.scala:158-159): one Program per aggregation
// argument (empty for count(*)), kinds CAPF_AGG_*
JNI(jlong, tableGroup)(JNIEnv *env, jobject, jlong t, jobjectArray by, jintArray kinds,
                       jobjectArray args, jbooleanArray distinct, jobjectArray names) {
  JStrs b(env, by), nm(env, names);
  std::vector<int32_t> k = ints(env, kinds), d = bools(env, distinct);
  Programs a(env, args);
  if (a.n() != (int32_t)k.size() || (int32_t)d.size() != (int32_t)k.size() || nm.n() != (int32_t)k.size()) {
    illegal_argument(env, "tableGroup: args, distinct and names need one entry per aggregation");
    return 0;
  }
  capf_table *out = nullptr;
  return fail(env, capf_table_group(T(t), b.n(), b.data(), (int32_t)k.size(), k.data(), a.data(),
                                    d.data(), nm.data(), &out))
             ? 0
             : H(out);
}
// group with the percentile fractions (capf_table_group_ex)
JNI(jlong, tableGroupEx)(JNIEnv *env, jobject, jlong t, jobjectArray by, jintArray kinds,
                         jobjectArray args, jbooleanArray distinct, jdoubleArray params, jobjectArray names) {
  JStrs b(env, by), nm(env, names);
  std::vector<int32_t> k = ints(env, kinds), d = bools(env, distinct);
  std::vector<double> p = doubles(env, params);
  Programs a(env, args);
  if (a.n() != (int32_t)k.size() || (int32_t)d.size() != (int32_t)k.size() || (int32_t)p.size() != (int32_t)k.size() ||
      nm.n() != (int32_t)k.size()) {
    illegal_argument(env, "tableGroupEx: args, distinct, params and names need one entry per aggregation");
    return 0;
  }
  capf_table *out = nullptr;
  return fail(env, capf_table_group_ex(T(t), b.n(), b.data(), (int32_t)k.size(), k.data(), a.data(),
                                       d.data(), p.data(), nm.data(), &out))
             ? 0
             : H(out);
}
// UNWIND (RelationalPlanner.scala:99-101): a literal / parameter list given as
// direct buffers (n elements, 8 or 1 bytes each; valid = n bytes or null)
JNI(jlong, tableExplodeValues)(JNIEnv *env, jobject, jlong t, jstring name, jint type, jlong n,
                               jobject values, jobject valid) {
  JStr nm(env, name);
  capf_table *out = nullptr;
  return fail(env, capf_table_explode_values(T(t), nm.p, type, n, values ? direct(env, values) : nullptr,
                                             valid ? (const uint8_t *)direct(env, valid) : nullptr, &out))
             ? 0
             : H(out);
}
JNI(jlong, tableExplodeList)(JNIEnv *env, jobject, jlong t, jstring list_col, jstring name) {
  JStr l(env, list_col), nm(env, name);
  capf_table *out = nullptr;
  return fail(env, capf_table_explode_list(T(t), l.p, nm.p, &out)) ? 0 : H(out);
}
// a LIST property column (CTList) from direct buffers: offsets (size + 1 int64),
// element values (8 B, BOOLEAN 1 B), list validity (size bytes) or null
JNI(jlong, tableAddList)(JNIEnv *env, jobject, jlong t, jstring name, jint elem_type, jobject offsets,
                         jobject values, jobject valid) {
  JStr nm(env, name);
  if (!offsets || !direct(env, offsets)) {
    illegal_argument(env, "tableAddList: offsets must be a direct buffer");
    return 0;
  }
  capf_table *out = nullptr;
  return fail(env, capf_table_add_list(T(t), nm.p, elem_type, (const int64_t *)direct(env, offsets),
                                       values ? direct(env, values) : nullptr,
                                       valid ? (const uint8_t *)direct(env, valid) : nullptr, &out))
             ? 0
             : H(out);
}
// labels(n) / keys(n) (FlinkSQLExprMapper.scala:136-153): a LIST<STRING> column
JNI(jlong, tableNameList)(JNIEnv *env, jobject, jlong t, jobjectArray cols, jintArray kinds, jlongArray codes,
                          jstring name) {
  JStrs c(env, cols);
  JStr nm(env, name);
  const std::vector<int32_t> k = ints(env, kinds);
  const std::vector<int64_t> cd = longs(env, codes);
  capf_table *out = nullptr;
  return fail(env, capf_table_name_list(T(t), (int32_t)k.size(), c.data(), k.data(), cd.data(), nm.p, &out)) ? 0
                                                                                                           : H(out);
}
// a list literal of per-row elements (FlinkSQLExprMapper.scala:71 array(...))
JNI(jlong, tableListColumns)(JNIEnv *env, jobject, jlong t, jobjectArray cols, jstring name) {
  JStrs c(env, cols);
  JStr nm(env, name);
  capf_table *out = nullptr;
  return fail(env, capf_table_list_columns(T(t), c.n(), c.data(), nm.p, &out)) ? 0 : H(out);
}
JNI(jlong, tableWithColumns)(JNIEnv *env, jobject, jlong t, jobjectArray exprs,
                             jobjectArray names) {  // Table.scala:170
  Programs e(env, exprs);
  JStrs nm(env, names);
  capf_table *out = nullptr;
  return fail(env, capf_table_with_columns(T(t), e.n(), e.data(), nm.data(), &out)) ? 0 : H(out);
}
JNI(void, tableShow)(JNIEnv *env, jobject, jlong t, jint rows) {  // Table.scala:177
  fail(env, capf_table_show(T(t), rows));
}

// ---------------------------------------------------------------- graph inputs
JNI(jlong, rmatRelTable)(JNIEnv *env, jobject, jlong s, jint scale, jlong seed, jint t_a,
                         jint t_ab, jint t_abc, jlong first, jlong count, jlong id_base,
                         jstring id_col, jstring src_col, jstring dst_col) {
  JStr i(env, id_col), a(env, src_col), b(env, dst_col);
  capf_table *out = nullptr;
  return fail(env, capf_rmat_rel_table(S(s), scale, (uint64_t)seed, (uint32_t)t_a, (uint32_t)t_ab,
                                       (uint32_t)t_abc, first, count, id_base, i.p, a.p, b.p,
                                       &out))
             ? 0
             : H(out);
}
JNI(jlong, rangeNodeTable)(JNIEnv *env, jobject, jlong s, jlong base, jlong n, jlong seed,
                           jstring id_col, jstring label_col) {
  JStr i(env, id_col), l(env, label_col);
  capf_table *out = nullptr;
  return fail(env, capf_range_node_table(S(s), base, n, (uint64_t)seed, i.p, l.p, &out)) ? 0
                                                                                          : H(out);
}
// EdgeListDataSource.graph (EdgeListDataSource.scala:56-92)
JNI(jlong, edgeListParse)(JNIEnv *env, jobject, jlong s, jobject bytes, jlong nbytes, jstring sep,
                          jstring comment, jstring id_col, jstring src_col, jstring dst_col) {
  JStr sp(env, sep), cm(env, comment), i(env, id_col), a(env, src_col), b(env, dst_col);
  capf_table *out = nullptr;
  return fail(env, capf_edge_list_parse(S(s), (const char *)direct(env, bytes), nbytes, sp.p, cm.p,
                                        i.p, a.p, b.p, &out))
             ? 0
             : H(out);
}
JNI(jlong, edgeListRead)(JNIEnv *env, jobject, jlong s, jstring path, jstring sep,
                         jstring comment, jstring id_col, jstring src_col, jstring dst_col) {
  JStr pa(env, path), sp(env, sep), cm(env, comment), i(env, id_col), a(env, src_col),
      b(env, dst_col);
  capf_table *out = nullptr;
  return fail(env, capf_edge_list_read(S(s), pa.p, sp.p, cm.p, i.p, a.p, b.p, &out)) ? 0 : H(out);
}

// ---------------------------------------------------------------- fused operators
// VarLengthExpand → Distinct → Aggregate (VarLengthExpandPlanner.scala:82-259)
JNI(jlong, varLengthReach)(JNIEnv *env, jobject, jlong s, jlong rels, jstring src_col,
                           jstring dst_col, jlong sources, jstring source_id, jlong targets,
                           jstring target_id, jint lower, jint upper, jstring out_source,
                           jstring out_reach) {
  JStr a(env, src_col), b(env, dst_col), si(env, source_id), ti(env, target_id),
      os(env, out_source), orr(env, out_reach);
  capf_table *out = nullptr;
  return fail(env, capf_var_length_reach(S(s), T(rels), a.p, b.p, T(sources), si.p, T(targets),
                                         ti.p, lower, upper, os.p, orr.p, &out))
             ? 0
             : H(out);
}

// ---------------------------------------------------------------- multi-GPU
JNI(jlong, tableNodePartition)(JNIEnv *env, jobject, jlong t, jstring key_col, jlong node_base,
                               jlong n_nodes, jint parts, jint part) {
  JStr k(env, key_col);
  capf_table *out = nullptr;
  return fail(env, capf_table_node_partition(T(t), k.p, node_base, n_nodes, parts, part, &out))
             ? 0
             : H(out);
}
JNI(void, chain2ShardedCount)(JNIEnv *env, jobject, jlong s, jlong in_copy, jstring in_dst,
                              jlong out_copy, jstring out_src, jstring out_dst, jlong node_base,
                              jlong n_nodes, jint parts, jint part, jlong d_partial) {
  JStr id(env, in_dst), os(env, out_src), od(env, out_dst);
  fail(env, capf_chain2_sharded_count(S(s), T(in_copy), id.p, T(out_copy), os.p, od.p, node_base,
                                      n_nodes, parts, part, reinterpret_cast<int64_t *>(d_partial)));
}
// 2-D out-copy: rows with both endpoints owned first (their count → nDiagOut[0])
JNI(jlong, tableNodePartitionDiag)(JNIEnv *env, jobject, jlong t, jstring src_col, jstring dst_col,
                                   jlong node_base, jlong n_nodes, jint parts, jint part,
                                   jlongArray nDiagOut) {
  JStr a(env, src_col), b(env, dst_col);
  capf_table *out = nullptr;
  int64_t nd = 0;
  if (fail(env, capf_table_node_partition_diag(T(t), a.p, b.p, node_base, n_nodes, parts, part, &out, &nd)))
    return 0;
  jlong v = nd;
  env->SetLongArrayRegion(nDiagOut, 0, 1, &v);
  return H(out);
}
JNI(void, chain2ShardedCountDiag)(JNIEnv *env, jobject, jlong s, jlong in_copy, jstring in_dst,
                                  jlong out_copy, jstring out_src, jstring out_dst, jlong n_diag,
                                  jlongArray hot_ids, jlong node_base, jlong n_nodes, jint parts,
                                  jint part, jlong d_partial) {
  JStr id(env, in_dst), os(env, out_src), od(env, out_dst);
  const jsize nh = hot_ids ? env->GetArrayLength(hot_ids) : 0;
  std::vector<int64_t> hot(nh > 0 ? nh : 1);
  if (nh > 0) {
    std::vector<jlong> h(nh);
    env->GetLongArrayRegion(hot_ids, 0, nh, h.data());
    for (jsize i = 0; i < nh; ++i) hot[i] = h[i];
  }
  fail(env, capf_chain2_sharded_count_diag(S(s), T(in_copy), id.p, T(out_copy), os.p, od.p, n_diag, nh,
                                           hot.data(), node_base, n_nodes, parts, part,
                                           reinterpret_cast<int64_t *>(d_partial)));
}
JNI(void, triangleCountPart)(JNIEnv *env, jobject, jlong s, jlong rels, jstring src_col,
                             jstring dst_col, jlong node_base, jlong n_nodes, jint parts,
                             jint part, jlong d_count) {
  JStr a(env, src_col), b(env, dst_col);
  fail(env, capf_triangle_count_part(S(s), T(rels), a.p, b.p, node_base, n_nodes, parts, part,
                                     reinterpret_cast<int64_t *>(d_count)));
}
JNI(jlong, chain2HistLen)(JNIEnv *, jobject, jlong n_nodes) { return capf_chain2_hist_len(n_nodes); }
JNI(jlong, chain2LocalHists)(JNIEnv *env, jobject, jlong s, jlong rels, jstring src_col,
                             jstring dst_col, jlong node_base, jlong n_nodes, jlong d_in,
                             jlong d_out) {
  JStr a(env, src_col), b(env, dst_col);
  int64_t loops = 0;
  fail(env, capf_chain2_local_hists(S(s), T(rels), a.p, b.p, node_base, n_nodes,
                                    reinterpret_cast<uint32_t *>(d_in),
                                    reinterpret_cast<uint32_t *>(d_out), &loops));
  return loops;
}
// FS graph source: all-LONG CSV tables parsed on the GPU
JNI(jlong, csvReadLongs)(JNIEnv *env, jobject, jlong s, jstring path, jstring sep, jobjectArray names) {
  JStr p(env, path), d(env, sep);
  JStrs nm(env, names);
  capf_table *out = nullptr;
  return fail(env, capf_csv_read_longs(S(s), p.p, d.p, nm.n(), nm.data(), &out)) ? 0 : H(out);
}
JNI(jlong, csvParseLongs)(JNIEnv *env, jobject, jlong s, jobject bytes, jlong nbytes, jstring sep,
                          jobjectArray names) {
  JStr d(env, sep);
  JStrs nm(env, names);
  capf_table *out = nullptr;
  return fail(env, capf_csv_parse_longs(S(s), (const char *)direct(env, bytes), nbytes, d.p, nm.n(),
                                        nm.data(), &out))
             ? 0
             : H(out);
}
// distributed Table layer: hash routing + device-side column copies; the
// JVM side moves the [off[p], off[p+1]) slices with its collective library
// (counts → countsOut[0..parts))
JNI(jlong, tableHashRoute)(JNIEnv *env, jobject, jlong t, jobjectArray keys, jint parts,
                           jlongArray countsOut) {
  JStrs k(env, keys);
  std::vector<int64_t> cnt(parts > 0 ? parts : 1);
  capf_table *out = nullptr;
  if (fail(env, capf_table_hash_route(T(t), k.n(), k.data(), parts, cnt.data(), &out))) return 0;
  std::vector<jlong> v(cnt.begin(), cnt.end());
  env->SetLongArrayRegion(countsOut, 0, parts, v.data());
  return H(out);
}
// exchange wire format (dist_table.py): out = {min, max, non_null}
JNI(void, tableColumnRange)(JNIEnv *env, jobject, jlong t, jstring col, jlongArray out) {
  JStr c(env, col);
  int64_t mn = 0, mx = 0, nn = 0;
  if (fail(env, capf_table_column_range(T(t), c.p, &mn, &mx, &nn))) return;
  jlong v[3] = {(jlong)mn, (jlong)mx, (jlong)nn};
  env->SetLongArrayRegion(out, 0, 3, v);
}
// returns the row bytes W; d_out = 0: only W
JNI(jint, tablePackRows)(JNIEnv *env, jobject, jlong t, jobjectArray cols, jintArray width, jlongArray base,
                         jintArray nullable, jlong d_out) {
  JStrs c(env, cols);
  std::vector<int32_t> w = ints(env, width), nl = ints(env, nullable);
  std::vector<int64_t> b = longs(env, base);
  if ((int64_t)w.size() != c.n() || (int64_t)b.size() != c.n() || (int64_t)nl.size() != c.n()) {
    illegal_argument(env, "tablePackRows: width, base and nullable need one entry per column");
    return 0;
  }
  int32_t W = 0;
  fail(env, capf_table_pack_rows(T(t), c.n(), c.data(), w.data(), b.data(), nl.data(), &W,
                                 reinterpret_cast<void *>(d_out)));
  return W;
}
JNI(jlong, tableFromPackedRows)(JNIEnv *env, jobject, jlong s, jobjectArray names, jintArray types,
                                jintArray width, jlongArray base, jintArray nullable, jlong d_rows, jlong nrows) {
  JStrs nm(env, names);
  std::vector<int32_t> ty = ints(env, types), w = ints(env, width), nl = ints(env, nullable);
  std::vector<int64_t> b = longs(env, base);
  if ((int64_t)ty.size() != nm.n() || (int64_t)w.size() != nm.n() || (int64_t)b.size() != nm.n() ||
      (int64_t)nl.size() != nm.n()) {
    illegal_argument(env, "tableFromPackedRows: types, width, base and nullable need one entry per column");
    return 0;
  }
  capf_table *out = nullptr;
  if (fail(env, capf_table_from_packed_rows(S(s), nm.n(), nm.data(), ty.data(), w.data(), b.data(), nl.data(),
                                            reinterpret_cast<const void *>(d_rows), nrows, &out)))
    return 0;
  return H(out);
}
JNI(void, tableDownloadDevice)(JNIEnv *env, jobject, jlong t, jstring col, jlong d_values,
                               jlong d_valid) {
  JStr c(env, col);
  fail(env, capf_table_download_device(T(t), c.p, reinterpret_cast<void *>(d_values),
                                       reinterpret_cast<uint8_t *>(d_valid)));
}
JNI(jboolean, tableHasNulls)(JNIEnv *env, jobject, jlong t, jstring col) {
  JStr c(env, col);
  int32_t h = 0;
  fail(env, capf_table_has_nulls(T(t), c.p, &h));
  return (jboolean)(h ? 1 : 0);
}
JNI(jlong, dotU32)(JNIEnv *env, jobject, jlong s, jlong d_a, jlong d_b, jlong n) {
  uint64_t r = 0;
  fail(env, capf_dot_u32(S(s), reinterpret_cast<const uint32_t *>(d_a),
                         reinterpret_cast<const uint32_t *>(d_b), n, &r));
  return (jlong)r;
}

// ------------------------------------------------ rank communicator (RCCL, capf_comm_*)
// the 128-byte unique id travels as a Java byte[] (rank 0 creates it, the
// launcher hands it to every rank)
JNI(jbyteArray, commUniqueId)(JNIEnv *env, jobject) {
  uint8_t id[CAPF_COMM_ID_BYTES];
  if (fail(env, capf_comm_unique_id(id))) return nullptr;
  jbyteArray a = env->NewByteArray(CAPF_COMM_ID_BYTES);
  env->SetByteArrayRegion(a, 0, CAPF_COMM_ID_BYTES, reinterpret_cast<const jbyte *>(id));
  return a;
}
JNI(jlong, commInit)(JNIEnv *env, jobject, jlong s, jint world, jint rank, jbyteArray id) {
  uint8_t raw[CAPF_COMM_ID_BYTES] = {0};
  if (!id || env->GetArrayLength(id) != CAPF_COMM_ID_BYTES) {
    illegal_argument(env, "commInit: the id must be 128 bytes");
    return 0;
  }
  env->GetByteArrayRegion(id, 0, CAPF_COMM_ID_BYTES, reinterpret_cast<jbyte *>(raw));
  capf_comm *c = nullptr;
  if (fail(env, capf_comm_init(S(s), world, rank, raw, &c))) return 0;
  return reinterpret_cast<jlong>(c);
}
JNI(void, commDestroy)(JNIEnv *env, jobject, jlong c) {
  fail(env, capf_comm_destroy(reinterpret_cast<capf_comm *>(c)));
}
JNI(void, commAllReduceI64)(JNIEnv *env, jobject, jlong c, jlong d_buf, jlong n, jint op) {
  fail(env, capf_comm_all_reduce_i64(reinterpret_cast<capf_comm *>(c), reinterpret_cast<int64_t *>(d_buf), n, op));
}
JNI(void, commAllGatherBytes)(JNIEnv *env, jobject, jlong c, jlong d_send, jlong bytes, jlong d_recv) {
  fail(env, capf_comm_all_gather_bytes(reinterpret_cast<capf_comm *>(c), reinterpret_cast<const void *>(d_send),
                                       bytes, reinterpret_cast<void *>(d_recv)));
}
JNI(void, commAllToAllBytes)(JNIEnv *env, jobject, jlong c, jlong d_send, jlongArray send_bytes, jlong d_recv,
                             jlongArray recv_bytes) {
  std::vector<int64_t> sb = longs(env, send_bytes), rb = longs(env, recv_bytes);
  int32_t rank = 0, world = 0;
  if (fail(env, capf_comm_rank(reinterpret_cast<capf_comm *>(c), &rank, &world))) return;
  if ((int32_t)sb.size() != world || (int32_t)rb.size() != world) {
    illegal_argument(env, "commAllToAllBytes: sendBytes and recvBytes need one entry per rank");
    return;
  }
  fail(env, capf_comm_all_to_all_bytes(reinterpret_cast<capf_comm *>(c), reinterpret_cast<const void *>(d_send),
                                       sb.data(), reinterpret_cast<void *>(d_recv), rb.data()));
}
JNI(jint, commRank)(JNIEnv *env, jobject, jlong c) {
  int32_t r = 0, w = 0;
  fail(env, capf_comm_rank(reinterpret_cast<capf_comm *>(c), &r, &w));
  return r;
}
JNI(jint, commWorld)(JNIEnv *env, jobject, jlong c) {
  int32_t r = 0, w = 0;
  fail(env, capf_comm_rank(reinterpret_cast<capf_comm *>(c), &r, &w));
  return w;
}
// device buffers of the session pool (exchange buffers, count slots)
JNI(jlong, sessionAlloc)(JNIEnv *env, jobject, jlong s, jlong bytes) {
  void *d = nullptr;
  if (fail(env, capf_session_alloc(S(s), bytes, &d))) return 0;
  return reinterpret_cast<jlong>(d);
}
JNI(void, sessionFree)(JNIEnv *env, jobject, jlong s, jlong d) {
  fail(env, capf_session_free(S(s), reinterpret_cast<void *>(d)));
}
// device ⇄ host through a direct buffer (kind 1 host → device, 2 device → host)
JNI(void, sessionCopy)(JNIEnv *env, jobject, jlong s, jlong d, jobject host, jlong bytes, jint kind) {
  void *h = direct(env, host);
  if (!h || bytes < 0 || env->GetDirectBufferCapacity(host) < bytes) {
    illegal_argument(env, "sessionCopy: a direct buffer of at least `bytes` bytes is required");
    return;
  }
  if (kind == 1) fail(env, capf_session_copy(S(s), reinterpret_cast<void *>(d), h, bytes, 1));
  else fail(env, capf_session_copy(S(s), h, reinterpret_cast<const void *>(d), bytes, 2));
}
// the session literal set of a long IN list (CAPF_OP_IN_SET): its id
JNI(jint, sessionLiteralSet)(JNIEnv *env, jobject, jlong s, jlongArray values) {
  const std::vector<int64_t> v = longs(env, values);
  int32_t id = -1;
  if (fail(env, capf_session_literal_set(S(s), v.data(), (int64_t)v.size(), &id))) return -1;
  return id;
}
// a code map of CAPF_OP_STR_MAP (codes[c] = the function's result code for string c): its id
JNI(jint, sessionCodeMap)(JNIEnv *env, jobject, jlong s, jlongArray codes) {
  const std::vector<int64_t> v = longs(env, codes);
  int32_t id = -1;
  if (fail(env, capf_session_code_map(S(s), v.data(), (int64_t)v.size(), &id))) return -1;
  return id;
}
// the code map `id` grown to the dictionary's current size: its id (the same one when replaced in place)
JNI(jint, sessionCodeMapExtend)(JNIEnv *env, jobject, jlong s, jint id, jlongArray codes) {
  const std::vector<int64_t> v = longs(env, codes);
  int32_t nid = -1;
  if (fail(env, capf_session_code_map_extend(S(s), id, v.data(), (int64_t)v.size(), &nid))) return -1;
  return nid;
}
// a value map of CAPF_OP_VALUE_MAP (sorted keys / key pairs → STRING codes): its id
JNI(jint, sessionValueMap)(JNIEnv *env, jobject, jlong s, jlongArray keys, jlongArray keys2, jlongArray codes) {
  const std::vector<int64_t> k = longs(env, keys), c = longs(env, codes);
  std::vector<int64_t> k2;
  if (keys2) k2 = longs(env, keys2);
  if (c.size() != k.size() || (keys2 && k2.size() != k.size())) {
    illegal_argument(env, "sessionValueMap: keys, keys2 and codes need the same length");
    return -1;
  }
  int32_t id = -1;
  if (fail(env, capf_session_value_map(S(s), k.data(), keys2 ? k2.data() : nullptr, c.data(), (int64_t)k.size(), &id)))
    return -1;
  return id;
}
// device → device
JNI(void, sessionCopyDevice)(JNIEnv *env, jobject, jlong s, jlong dst, jlong src, jlong bytes) {
  fail(env, capf_session_copy(S(s), reinterpret_cast<void *>(dst), reinterpret_cast<const void *>(src), bytes, 3));
}
