// pip_buf_layout.h -- read-only view of a pip_buf chain segment.
//
// pip's checksum reads a chain only through pip_buf::payload(),
// payload_len(), total_len() and next() (pip/pip_checksum.cpp:140,145-146;
// accessors at pip/pip_buf.h:67-79).  pip_buf is header-only, so its object
// layout IS the ABI the drop-in has to honour.  With libstdc++ (pip's only
// toolchain on Linux) the members of pip/pip_buf.h:13-19 lie at:
//
//   enable_shared_from_this<pip_buf>::_M_weak_this   weak_ptr   0   (16 B)
//   void*      _payload                                         16
//   pip_uint32 _payload_len                                     24
//   pip_uint8  _is_alloc                                        28
//   pip_uint32 _total_len                                       32
//   weak_ptr<pip_buf>   _prev                                   40  (16 B)
//   shared_ptr<pip_buf> _next  (element pointer first)          56  (16 B)
//
// The link-substitution test (tests/test_boundary.py) runs pip's real stack,
// compiled from the reference's own pip_buf.h, against this view.
#ifndef PIP_BUF_LAYOUT_H
#define PIP_BUF_LAYOUT_H

#include <stddef.h>
#include <stdint.h>

struct pip_buf_layout {
    void* weak_this[2];
    void* payload;
    uint32_t payload_len;
    uint8_t is_alloc;
    uint32_t total_len;
    void* prev[2];
    const pip_buf_layout* next;
    void* next_ctrl;
};

static_assert(offsetof(pip_buf_layout, payload) == 16, "pip_buf::_payload offset");
static_assert(offsetof(pip_buf_layout, payload_len) == 24, "pip_buf::_payload_len offset");
static_assert(offsetof(pip_buf_layout, total_len) == 32, "pip_buf::_total_len offset");
static_assert(offsetof(pip_buf_layout, next) == 56, "pip_buf::_next offset");
static_assert(sizeof(pip_buf_layout) == 72, "sizeof(pip_buf)");

#endif
