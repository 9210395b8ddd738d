"""Drop-in replacement of the reference's `core` ASR modules (asr_engine, hardware_accel,
hotword_context) backed by libzasr.so on MI355X."""
