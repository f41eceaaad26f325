/* Links the gfx950 code object into libvcrt.so (the LOAD_SHADER_FROM_MEMORY analogue). */
    .section .rodata
    .balign 4096
    .globl vcrt_embedded_code_object
    .type vcrt_embedded_code_object, @object
vcrt_embedded_code_object:
    .incbin VCRT_CODE_OBJECT
    .globl vcrt_embedded_code_object_end
vcrt_embedded_code_object_end:
    .byte 0
    .section .note.GNU-stack,"",@progbits
