// Test infrastructure (not product code): a minimal in-process stand-in for the
// JVM side of JNI, so the adapter integration/jni/capf_jni.cpp can be BUILT and
// EXECUTED in this JDK-less image.
//
// It defines the JNIEnv member functions that tests/jni_stub/jni.h declares
// (the JNI specification's "JNI Functions": strings, primitive / object
// arrays, fields, direct buffers, exceptions) over a small object model, and
// exports a C API (fj_*) through which tests/jni_route.py builds Java objects
// (String, String[], long[], direct ByteBuffers, org.opencypher.gpu.Program …),
// calls the adapter's Java_org_opencypher_gpu_Native_00024_* symbols and reads
// back results and pending exceptions.  Semantics follow the JNI spec where
// the adapter can observe them: Get<Type>ArrayRegion outside the array throws
// ArrayIndexOutOfBoundsException, GetDirectBufferAddress of a non-direct
// object is NULL and its capacity -1, Throw / ThrowNew leave the exception
// pending until the caller (the "JVM") collects it.
#include <jni.h>

#include <cstdarg>
#include <cstdint>
#include <cstring>
#include <map>
#include <memory>
#include <string>
#include <vector>

namespace {

enum Kind { K_CLASS, K_STRING, K_INTS, K_LONGS, K_DOUBLES, K_BOOLS, K_BYTES, K_OBJECTS, K_DIRECT, K_OBJECT,
            K_THROWABLE };

struct Obj {
  Kind kind;
  std::string cls;  // class name (JNI form, a/b/C)
  std::string s;    // String value / Throwable message
  std::vector<int32_t> i32;
  std::vector<int64_t> i64;
  std::vector<double> f64;
  std::vector<uint8_t> u8;
  std::vector<Obj *> objs;
  void *addr = nullptr;  // direct buffer
  int64_t cap = -1;
  int32_t code = 0;  // CapfNativeException kind
  std::map<std::string, Obj *> fields;
};

std::vector<std::unique_ptr<Obj>> arena;  // every object lives until fj_reset
std::map<std::string, Obj *> classes;
std::map<std::string, std::unique_ptr<std::string>> field_ids;
Obj *pending = nullptr;  // the pending exception
int64_t calls = 0;       // JNI functions called (a liveness check for the tests)
JNIEnv the_env;

Obj *make(Kind k, const std::string &cls) {
  arena.emplace_back(new Obj());
  Obj *o = arena.back().get();
  o->kind = k;
  o->cls = cls;
  return o;
}

Obj *O(jobject o) { return reinterpret_cast<Obj *>(o); }
template <class T>
T J(Obj *o) {
  return reinterpret_cast<T>(o);
}

Obj *klass(const std::string &name) {
  auto it = classes.find(name);
  if (it != classes.end()) return it->second;
  Obj *c = make(K_CLASS, name);
  classes[name] = c;
  return c;
}

void throw_new(const std::string &cls, const std::string &msg) {
  if (pending) return;  // the first exception stays pending
  Obj *t = make(K_THROWABLE, cls);
  t->s = msg;
  pending = t;
}

size_t length(Obj *o) {
  switch (o->kind) {
    case K_INTS: return o->i32.size();
    case K_LONGS: return o->i64.size();
    case K_DOUBLES: return o->f64.size();
    case K_BOOLS: case K_BYTES: return o->u8.size();
    case K_OBJECTS: return o->objs.size();
    default: return 0;
  }
}

bool in_range(Obj *o, jsize start, jsize len) {
  if (!o || start < 0 || len < 0 || (size_t)start + (size_t)len > length(o)) {
    throw_new("java/lang/ArrayIndexOutOfBoundsException", "array region out of bounds");
    return false;
  }
  return true;
}

}  // namespace

// ------------------------------------------------------------ JNIEnv (JNI spec)
jclass JNIEnv::FindClass(const char *name) {
  ++calls;
  return J<jclass>(klass(name));
}
jclass JNIEnv::GetObjectClass(jobject obj) {
  ++calls;
  return J<jclass>(klass(O(obj)->cls));
}
jmethodID JNIEnv::GetMethodID(jclass, const char *, const char *) {
  ++calls;
  return reinterpret_cast<jmethodID>(&the_env);  // constructors only; any non-NULL id
}
jfieldID JNIEnv::GetFieldID(jclass, const char *name, const char *) {
  ++calls;
  auto &p = field_ids[name];
  if (!p) p.reset(new std::string(name));
  return reinterpret_cast<jfieldID>(p.get());
}
jobject JNIEnv::GetObjectField(jobject obj, jfieldID field) {
  ++calls;
  const std::string &nm = *reinterpret_cast<std::string *>(field);
  auto it = O(obj)->fields.find(nm);
  return it == O(obj)->fields.end() ? nullptr : J<jobject>(it->second);
}
jobject JNIEnv::NewObject(jclass clazz, jmethodID ctor, ...) {
  ++calls;
  // the one constructor the adapter calls: CapfNativeException(int kind, String message)
  va_list ap;
  va_start(ap, ctor);
  jint kind = va_arg(ap, jint);
  jstring msg = va_arg(ap, jstring);
  va_end(ap);
  Obj *t = make(K_THROWABLE, O(clazz)->cls);
  t->code = kind;
  t->s = msg ? O(msg)->s : "";
  return J<jobject>(t);
}
jint JNIEnv::Throw(jthrowable obj) {
  ++calls;
  if (!pending) pending = O(obj);
  return 0;
}
jint JNIEnv::ThrowNew(jclass clazz, const char *message) {
  ++calls;
  throw_new(O(clazz)->cls, message ? message : "");
  return 0;
}
jstring JNIEnv::NewStringUTF(const char *utf) {
  ++calls;
  Obj *s = make(K_STRING, "java/lang/String");
  s->s = utf ? utf : "";
  return J<jstring>(s);
}
const char *JNIEnv::GetStringUTFChars(jstring str, jboolean *is_copy) {
  ++calls;
  if (is_copy) *is_copy = 0;
  return O(str)->s.c_str();
}
void JNIEnv::ReleaseStringUTFChars(jstring, const char *) { ++calls; }
jsize JNIEnv::GetArrayLength(jarray array) {
  ++calls;
  return (jsize)length(O(array));
}
jobjectArray JNIEnv::NewObjectArray(jsize len, jclass clazz, jobject init) {
  ++calls;
  Obj *a = make(K_OBJECTS, "[L" + O(clazz)->cls + ";");
  a->objs.assign(len, O(init));
  return J<jobjectArray>(a);
}
jobject JNIEnv::GetObjectArrayElement(jobjectArray array, jsize index) {
  ++calls;
  if (!in_range(O(array), index, 1)) return nullptr;
  return J<jobject>(O(array)->objs[index]);
}
void JNIEnv::SetObjectArrayElement(jobjectArray array, jsize index, jobject val) {
  ++calls;
  if (in_range(O(array), index, 1)) O(array)->objs[index] = O(val);
}
void JNIEnv::GetIntArrayRegion(jintArray array, jsize start, jsize len, jint *buf) {
  ++calls;
  if (in_range(O(array), start, len) && len) memcpy(buf, O(array)->i32.data() + start, len * sizeof(jint));
}
void JNIEnv::GetLongArrayRegion(jlongArray array, jsize start, jsize len, jlong *buf) {
  ++calls;
  if (in_range(O(array), start, len) && len) memcpy(buf, O(array)->i64.data() + start, len * sizeof(jlong));
}
void JNIEnv::GetDoubleArrayRegion(jdoubleArray array, jsize start, jsize len, jdouble *buf) {
  ++calls;
  if (in_range(O(array), start, len) && len) memcpy(buf, O(array)->f64.data() + start, len * sizeof(jdouble));
}
void JNIEnv::GetBooleanArrayRegion(jbooleanArray array, jsize start, jsize len, jboolean *buf) {
  ++calls;
  if (in_range(O(array), start, len) && len) memcpy(buf, O(array)->u8.data() + start, len);
}
void JNIEnv::SetLongArrayRegion(jlongArray array, jsize start, jsize len, const jlong *buf) {
  ++calls;
  if (in_range(O(array), start, len) && len) memcpy(O(array)->i64.data() + start, buf, len * sizeof(jlong));
}
void JNIEnv::SetDoubleArrayRegion(jdoubleArray array, jsize start, jsize len, const jdouble *buf) {
  ++calls;
  if (in_range(O(array), start, len) && len) memcpy(O(array)->f64.data() + start, buf, len * sizeof(jdouble));
}
jbyteArray JNIEnv::NewByteArray(jsize len) {
  ++calls;
  Obj *a = make(K_BYTES, "[B");
  a->u8.assign(len, 0);
  return J<jbyteArray>(a);
}
void JNIEnv::GetByteArrayRegion(jbyteArray array, jsize start, jsize len, jbyte *buf) {
  ++calls;
  if (in_range(O(array), start, len) && len) memcpy(buf, O(array)->u8.data() + start, len);
}
void JNIEnv::SetByteArrayRegion(jbyteArray array, jsize start, jsize len, const jbyte *buf) {
  ++calls;
  if (in_range(O(array), start, len) && len) memcpy(O(array)->u8.data() + start, buf, len);
}
void *JNIEnv::GetDirectBufferAddress(jobject buf) {
  ++calls;
  return O(buf)->kind == K_DIRECT ? O(buf)->addr : nullptr;
}
jlong JNIEnv::GetDirectBufferCapacity(jobject buf) {
  ++calls;
  return O(buf)->kind == K_DIRECT ? O(buf)->cap : -1;
}
void JNIEnv::DeleteLocalRef(jobject) { ++calls; }

// ------------------------------------------------------------ C API for the tests
extern "C" {
JNIEXPORT void *fj_env() { return &the_env; }
JNIEXPORT void fj_reset() {
  arena.clear();
  classes.clear();
  pending = nullptr;
}
JNIEXPORT int64_t fj_calls() { return calls; }
JNIEXPORT void *fj_string(const char *s) {
  Obj *o = make(K_STRING, "java/lang/String");
  o->s = s ? s : "";
  return o;
}
JNIEXPORT const char *fj_string_value(void *o) { return o ? O((jobject)o)->s.c_str() : nullptr; }
JNIEXPORT void *fj_ints(const int32_t *v, int64_t n) {
  Obj *o = make(K_INTS, "[I");
  o->i32.assign(v, v + n);
  return o;
}
JNIEXPORT void *fj_longs(const int64_t *v, int64_t n) {
  Obj *o = make(K_LONGS, "[J");
  if (v) o->i64.assign(v, v + n);
  else o->i64.assign(n, 0);
  return o;
}
JNIEXPORT void *fj_doubles(const double *v, int64_t n) {
  Obj *o = make(K_DOUBLES, "[D");
  if (v) o->f64.assign(v, v + n);
  else o->f64.assign(n, 0.0);
  return o;
}
JNIEXPORT void *fj_bools(const uint8_t *v, int64_t n) {
  Obj *o = make(K_BOOLS, "[Z");
  o->u8.assign(v, v + n);
  return o;
}
JNIEXPORT void *fj_bytes(const uint8_t *v, int64_t n) {
  Obj *o = make(K_BYTES, "[B");
  o->u8.assign(v, v + n);
  return o;
}
JNIEXPORT void *fj_objects(void *const *items, int64_t n, const char *cls) {
  Obj *o = make(K_OBJECTS, std::string("[L") + cls + ";");
  for (int64_t i = 0; i < n; ++i) o->objs.push_back(O((jobject)items[i]));
  return o;
}
JNIEXPORT void *fj_direct(void *addr, int64_t cap) {  // java.nio.DirectByteBuffer
  Obj *o = make(K_DIRECT, "java/nio/DirectByteBuffer");
  o->addr = addr;
  o->cap = cap;
  return o;
}
JNIEXPORT void *fj_heap_buffer() {  // java.nio.HeapByteBuffer: not direct
  return make(K_OBJECT, "java/nio/HeapByteBuffer");
}
// org.opencypher.gpu.Program(ops: int[], iargs: long[], fargs: double[], names: String[])
JNIEXPORT void *fj_program(void *ops, void *iargs, void *fargs, void *names) {
  Obj *o = make(K_OBJECT, "org/opencypher/gpu/Program");
  o->fields["ops"] = O((jobject)ops);
  o->fields["iargs"] = O((jobject)iargs);
  o->fields["fargs"] = O((jobject)fargs);
  o->fields["names"] = O((jobject)names);
  return o;
}
JNIEXPORT int64_t fj_length(void *o) { return o ? (int64_t)length(O((jobject)o)) : -1; }
JNIEXPORT void *fj_element(void *o, int64_t i) { return O((jobject)o)->objs[i]; }
JNIEXPORT void fj_get_longs(void *o, int64_t *out) {
  auto &v = O((jobject)o)->i64;
  if (!v.empty()) memcpy(out, v.data(), v.size() * sizeof(int64_t));
}
JNIEXPORT void fj_get_doubles(void *o, double *out) {
  auto &v = O((jobject)o)->f64;
  if (!v.empty()) memcpy(out, v.data(), v.size() * sizeof(double));
}
JNIEXPORT void fj_get_bytes(void *o, uint8_t *out) {
  auto &v = O((jobject)o)->u8;
  if (!v.empty()) memcpy(out, v.data(), v.size());
}
// the pending exception (returns 0 if none; else 1 and clears it): its class,
// message and, for CapfNativeException, the capf status kind
JNIEXPORT int fj_take_exception(const char **cls, const char **msg, int32_t *code) {
  if (!pending) return 0;
  static std::string c, m;
  c = pending->cls;
  m = pending->s;
  *cls = c.c_str();
  *msg = m.c_str();
  *code = pending->code;
  pending = nullptr;
  return 1;
}
}
