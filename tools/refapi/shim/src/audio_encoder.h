// Forwarding header (see shim/src/text_decoder.h): "../src/audio_encoder.h" -> include/audio_encoder.h
#pragma once
#include <audio_encoder.h>   // (angle brackets: the -I path, not this file's directory)
