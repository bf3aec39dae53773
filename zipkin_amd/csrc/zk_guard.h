// zk_guard.h — no C++ exception crosses the C ABI (every include/*.h: "never throws or aborts").
// A host allocation failure becomes ZK_ERR_CAPACITY, anything else ZK_ERR_INVALID_ARG.
#pragma once
#include <new>

#define ZK_GUARD_BEGIN try {
#define ZK_GUARD_END                          \
    }                                         \
    catch (const std::bad_alloc&) {           \
        return ZK_ERR_CAPACITY;               \
    }                                         \
    catch (...) {                             \
        return ZK_ERR_INVALID_ARG;            \
    }
