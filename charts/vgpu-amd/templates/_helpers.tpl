{{- define "vgpu.name" -}}
{{- default .Chart.Name .Values.nameOverride | trunc 63 | trimSuffix "-" -}}
{{- end -}}

{{- define "vgpu.fullname" -}}
{{- if .Values.fullnameOverride -}}
{{- .Values.fullnameOverride | trunc 63 | trimSuffix "-" -}}
{{- else -}}
{{- printf "%s-%s" .Release.Name (include "vgpu.name" .) | trunc 63 | trimSuffix "-" -}}
{{- end -}}
{{- end -}}

{{- define "vgpu.scheduler" -}}{{ include "vgpu.fullname" . }}-scheduler{{- end -}}
{{- define "vgpu.device-plugin" -}}{{ include "vgpu.fullname" . }}-device-plugin{{- end -}}
{{- define "vgpu.scheduler.tls" -}}{{ include "vgpu.scheduler" . }}-tls{{- end -}}

{{- define "vgpu.labels" -}}
app.kubernetes.io/name: {{ include "vgpu.name" . }}
app.kubernetes.io/instance: {{ .Release.Name }}
app.kubernetes.io/version: {{ .Values.version | quote }}
{{- with .Values.global.labels }}
{{ toYaml . }}
{{- end }}
{{- end -}}
