// ck_zero.cpp -- MEASUREMENT ONLY: the six pip_checksum symbols returning 0, linked into
// pip's stack (without pip_checksum.o) as _ref/stack_tx_zero.  Its packets carry wrong
// checksums; it exists to time pip's TX path with no checksum work at all -- the ceiling
// any checksum offload of that path can approach (oracle/stack_tx_bench.cpp).
#include <netinet/in.h>
#include <stdint.h>

#include <memory>

class pip_buf;
uint32_t pip_fold_uint32(uint32_t n) { return n; }
uint32_t pip_standard_checksum(const void*, uint32_t, uint32_t s) { return s; }
uint16_t pip_ip_checksum(const void*, uint32_t) { return 0; }
uint16_t pip_inet_checksum(const void*, uint8_t, struct in_addr, struct in_addr, uint16_t) { return 0; }
uint16_t pip_inet6_checksum(const void*, uint8_t, struct in6_addr, struct in6_addr, uint16_t) { return 0; }
uint16_t pip_inet_checksum_buf(std::shared_ptr<pip_buf>, uint8_t, struct in_addr, struct in_addr) { return 0; }
uint16_t pip_inet6_checksum_buf(std::shared_ptr<pip_buf>, uint8_t, struct in6_addr, struct in6_addr) { return 0; }
