// Forwarding header (see shim/src/text_decoder.h): "../src/audio_injection.h" -> include/audio_injection.h
#pragma once
#include <audio_injection.h>   // (angle brackets: the -I path, not this file's directory)
