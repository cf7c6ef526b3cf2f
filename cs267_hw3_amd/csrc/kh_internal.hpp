// kh_internal.hpp — symbols shared between the library's translation units (not part of the ABI).
#pragma once

// Sets the thread-local message returned by kh_last_error().
void kh_set_error_internal(const char* msg);
