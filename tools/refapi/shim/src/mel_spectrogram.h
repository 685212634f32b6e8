// Forwarding header (see shim/src/text_decoder.h): "../src/mel_spectrogram.h" -> include/mel_spectrogram.h
#pragma once
#include <mel_spectrogram.h>   // (angle brackets: the -I path, not this file's directory)
