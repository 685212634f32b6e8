// Forwarding header for reference sources that name "../src/text_decoder.h"
// (tests/test_decoder_last_pos.cpp, test_decoder_no_audio.cpp): with
// tools/refapi/Makefile's -I shim/tests -I- that path resolves here, and from
// here to include/text_decoder.h.
#pragma once
#include <text_decoder.h>   // (angle brackets: the -I path, not this file's directory)
