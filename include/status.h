/* status.h -- status codes of the monotonic RNN-T C ABI.
 * Same enumerators and values as the reference (include/status.h:4-10), so callers that switch on
 * them keep working; the message table follows status.h:17-29 with the GPU wording made HIP-neutral. */
#ifndef MONOTONIC_RNNT_STATUS_H
#define MONOTONIC_RNNT_STATUS_H

typedef enum {
    RNNT_STATUS_SUCCESS = 0,
    RNNT_STATUS_MEMOPS_FAILED = 1,
    RNNT_STATUS_INVALID_VALUE = 2,
    RNNT_STATUS_EXECUTION_FAILED = 3,
    RNNT_STATUS_UNKNOWN_ERROR = 4
} RNNTStatus;

#ifdef __cplusplus
inline
#else
static inline
#endif
const char *rnntGetStatusString(RNNTStatus status) {
    switch (status) {
        case RNNT_STATUS_SUCCESS:
            return "no error";
        case RNNT_STATUS_MEMOPS_FAILED:
            return "device memcpy or memset failed";
        case RNNT_STATUS_INVALID_VALUE:
            return "invalid value";
        case RNNT_STATUS_EXECUTION_FAILED:
            return "execution failed";
        case RNNT_STATUS_UNKNOWN_ERROR:
        default:
            return "unknown error";
    }
}

#endif /* MONOTONIC_RNNT_STATUS_H */
