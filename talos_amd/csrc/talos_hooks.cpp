// talos_hooks.cpp — TaLoS's TLS-processing interface, implemented by libtlsgpu
// with the reference's exact signatures
// (src/talos/enclaveshim/tls_processing_interface.h:23-49,
//  tls_processing_interface.c:29-90):
//
//   public  tls_processing_register_{ssl_read,ssl_write}_processing_cb,
//           tls_processing_register_{set_ssl_type,new_connection,free_connection}_cb
//   private tls_processing_ssl_read / _ssl_write  (called by the TaLoS-patched
//           ssl3_read_bytes / do_ssl3_write, s3_pkt.c.patch:39-52, 19-33),
//           tls_processing_set_ssl_type / _new_connection / _free_connection
//           (bio_lib.c.patch, ssl_lib.c.patch),
//           ecall_tls_processing_module_init (TaLoS's initialize_library ->
//           the module's tls_processing_module_init, enclaveshim_ecalls.c:440)
//
// so an existing TaLoS module (logpoint.c:127-135 style) registers against the
// engine unchanged.  The registered read/write callbacks fire
//   * from the TaLoS-patched record layer when libtlsgpu.so is interposed
//     (its calls to tls_processing_* bind here), and
//   * from the engine's own host-delivery paths (engine.cpp: tlsgpu_open_host /
//     tlsgpu_seal_host, tlsgpu_deliver_host for the batch and wire paths,
//     tlsgpu_hook_write_streams), with the SSL* the caller associated with each
//     session (tlsgpu_sessions_set_owner).
//
// Length argument: the patched s3_pkt.c declares and calls
// tls_processing_ssl_read/_write with `unsigned int len` BY VALUE
// (s3_pkt.c.patch:13-14, :31, :48), while the interface takes `unsigned int
// *len` and hands it to the callback, which logpoint-style modules
// dereference: the reference's nosgx build crashes as soon as such a module is
// registered (reproduced by tests/test_talos_hooks.py with the CPU build).
// What tls_processing_ssl_read/_write make of their third argument is a
// process-wide setting, TLSGPU_TALOS_LEN (read once at load):
//   "value"   — always the by-value length: the low 32 bits of the argument
//               (the upper half of a 32-bit argument register is undefined in
//               the x86-64 SysV ABI, so only the low half is read).  For the
//               TaLoS-patched record layer.
//   "pointer" — always a pointer (the interface as declared).
//   unset / "auto" — a "pointer" whose value is below 64 KiB (never a mapped
//               user address, vm.mmap_min_addr; a TLS record length is <= 18
//               KiB) is taken as the length.  This relies on the caller
//               zero-extending the 32-bit length into the register, which gcc
//               and clang do in practice but the ABI does not promise: set
//               "value" for a patched tree built by another compiler.
// The engine's own host-delivery paths (tg::talos_read / talos_write below)
// always pass real pointers and are not affected by the setting.
#include <dlfcn.h>

#include <atomic>
#include <cstdint>
#include <cstdlib>
#include <cstring>

#include "tlsgpu_internal.h"

typedef struct ssl_st SSL;

namespace {
using rw_cb = void (*)(const SSL*, char*, unsigned int*);
using type_cb = void (*)(const void*, const long);
using conn_cb = void (*)(const SSL*);

std::atomic<rw_cb> g_read{nullptr}, g_write{nullptr};
std::atomic<type_cb> g_type{nullptr};
std::atomic<conn_cb> g_new{nullptr}, g_free{nullptr};
std::atomic<uint64_t> g_read_calls{0}, g_write_calls{0};

enum LenMode { LEN_AUTO, LEN_VALUE, LEN_POINTER };
const LenMode g_len_mode = [] {
  const char* v = getenv("TLSGPU_TALOS_LEN");
  if (v && !strcmp(v, "value")) return LEN_VALUE;
  if (v && !strcmp(v, "pointer")) return LEN_POINTER;
  return LEN_AUTO;
}();

// external: a call from the (patched) record layer, whose third argument may
// be the by-value length (see above); the engine's own calls pass pointers.
void call_rw(rw_cb cb, const SSL* s, char* data, unsigned int* len, bool external) {
  if (!cb) return;
  const uintptr_t v = reinterpret_cast<uintptr_t>(len);
  if (external && (g_len_mode == LEN_VALUE || (g_len_mode == LEN_AUTO && v < 65536))) {
    unsigned int n = static_cast<unsigned int>(v & 0xFFFFFFFFu);
    cb(s, data, &n);
  } else {
    cb(s, data, len);
  }
}
}  // namespace

extern "C" {
void tls_processing_register_ssl_read_processing_cb(rw_cb cb) { g_read.store(cb); }
void tls_processing_register_ssl_write_processing_cb(rw_cb cb) { g_write.store(cb); }
void tls_processing_register_set_ssl_type_cb(type_cb cb) { g_type.store(cb); }
void tls_processing_register_new_connection_cb(conn_cb cb) { g_new.store(cb); }
void tls_processing_register_free_connection_cb(conn_cb cb) { g_free.store(cb); }

void ecall_tls_processing_module_init(void) {
  // the module is linked into the application or the TaLoS library, not here
  auto init = reinterpret_cast<void (*)(void)>(dlsym(RTLD_DEFAULT, "tls_processing_module_init"));
  if (init) init();
}

void tls_processing_ssl_read(const SSL* s, char* data, unsigned int* len) {
  g_read_calls.fetch_add(1, std::memory_order_relaxed);
  call_rw(g_read.load(), s, data, len, true);
}
void tls_processing_ssl_write(const SSL* s, char* data, unsigned int* len) {
  g_write_calls.fetch_add(1, std::memory_order_relaxed);
  call_rw(g_write.load(), s, data, len, true);
}
void tls_processing_set_ssl_type(const void* b, const long type) {
  if (type_cb cb = g_type.load()) cb(b, type);
}
void tls_processing_new_connection(const SSL* s) {
  if (conn_cb cb = g_new.load()) cb(s);
}
void tls_processing_free_connection(const SSL* s) {
  if (conn_cb cb = g_free.load()) cb(s);
}

// read / write hook invocations since load, from any caller (include/tlsgpu.h)
int tlsgpu_talos_hook_stats(uint64_t* read_calls, uint64_t* write_calls) {
  if (read_calls) *read_calls = g_read_calls.load();
  if (write_calls) *write_calls = g_write_calls.load();
  return 0;
}
}  // extern "C"

namespace tg {
bool talos_read_hooked() { return g_read.load() != nullptr; }
bool talos_write_hooked() { return g_write.load() != nullptr; }
void talos_read(const void* ssl, uint8_t* data, uint32_t* len) {
  g_read_calls.fetch_add(1, std::memory_order_relaxed);
  call_rw(g_read.load(), static_cast<const SSL*>(ssl), reinterpret_cast<char*>(data), len, false);
}
void talos_write(const void* ssl, uint8_t* data, uint32_t* len) {
  g_write_calls.fetch_add(1, std::memory_order_relaxed);
  call_rw(g_write.load(), static_cast<const SSL*>(ssl), reinterpret_cast<char*>(data), len, false);
}
}  // namespace tg
